// Probe (tuning only): k_pinf_find variants on one zlib stream read from a file, timed with HIP events.
//   hipcc -O3 --offload-arch=gfx950 -I reductionist-rs_amd/csrc tools/probe_pinf_find.hip -o tools/probe_pinf_find
//   tools/probe_pinf_find stream.zlib
// variant 0: the product kernel; 1: stop after the cheap BTYPE/HLIT/HDIST test; 2: after the code-length
// code's completeness; 3: no stored test.
#define RDX_PINF_FIND_VARIANTS 1
#include "../reductionist-rs_amd/csrc/k_pinflate.hip"

#include <cstdio>
#include <vector>

using namespace rdx;

namespace rdx {
namespace {
__global__ __launch_bounds__(256) void k_find_var(PinfArgs a, int variant, unsigned long long *ctr) {
    __shared__ uint32_t win[kFindWin];
    Stream S = make_stream(a);
    const uint64_t q0 = a.first_byte + (uint64_t)blockIdx.x * kFindBytes;
    S.stage(win, kFindWin, q0 >> 2, a.nw);
    unsigned long long c = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t q = q0 + threadIdx.x + 256 * k;
        if (q >= a.end_byte) break;
        const uint32_t w = S.at(8 * q);
        for (uint32_t b = 0; b < 8; ++b) {
            if (((w >> (b + 1)) & 3) != 2) continue;
            const uint64_t p = 8 * q + b;
            if (variant == 1) {
                const uint32_t h = S.at(p);
                c += ((h >> 3) & 31) <= 29 && ((h >> 8) & 31) <= 29;
                continue;
            }
            if (variant == 2) {
                const uint32_t h = S.at(p);
                if (((h >> 3) & 31) > 29 || ((h >> 8) & 31) > 29) continue;
                const uint32_t nc = ((h >> 13) & 15) + 4;
                uint64_t cb = (uint64_t)S.at(p + 17) | (uint64_t)S.at(p + 49) << 32;
                cb &= (1ull << (3 * nc)) - 1;
                uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                for (int i = 0; i < 19; ++i) {
                    const uint32_t l = (uint32_t)(cb >> (3 * i)) & 7;
#pragma unroll
                    for (int qq = 1; qq < 8; ++qq) cnt[qq] += l == (uint32_t)qq ? 1u : 0u;
                }
                int left = 1;
#pragma unroll
                for (int l = 1; l < 8; ++l) left = (left << 1) - (int)cnt[l];
                c += left == 0;
                continue;
            }
            c += dyn_candidate(S, p, a.end_bits);
        }
        if (variant != 3 && q >= a.first_byte + 1 && q + 4 <= a.end_byte) {
            const uint32_t v = S.at(8 * q - 8);
            const uint32_t len = (v >> 8) & 0xffff;
            const uint32_t nlen = S.at(8 * q + 16) & 0xffff;
            c += len == (~nlen & 0xffff) && ((v >> 6) & 3) == 0 && q + 4 + len <= a.end_byte;
        }
    }
    if (c) atomicAdd(ctr, c);
}
}  // namespace
}  // namespace rdx

int main(int argc, char **argv) {
    FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 1;
    std::vector<uint8_t> in(1 << 26);
    const size_t n = std::fread(in.data(), 1, in.size(), f);
    std::fclose(f);
    uint8_t *d = nullptr;
    hipMalloc(&d, n + 16);
    hipMemcpy(d, in.data(), n, hipMemcpyHostToDevice);
    PinfArgs a{};
    a.w = reinterpret_cast<const uint32_t *>(d);
    a.first_byte = 0;
    a.end_byte = n;
    a.end_bits = 8 * n;
    a.nw = (n + 3) / 4;
    a.lmask = n % 4 ? (1u << (8 * (n % 4))) - 1 : 0xffffffffu;
    unsigned long long *ctr = nullptr;
    hipMalloc(&ctr, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const uint32_t grid = (uint32_t)((n + kFindBytes - 1) / kFindBytes);
    {   // the product kernel
        PinfState *stt = nullptr;
        uint64_t *cand = nullptr;
        hipMalloc(&stt, sizeof(PinfState));
        hipMalloc(&cand, 8 * kPinfMaxCand);
        a.state = stt;
        a.cand = cand;
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(stt, 0, sizeof(PinfState));
            hipEventRecord(e0, 0);
            launch_pinf_find(a, 0);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            PinfState h{};
            hipMemcpy(&h, stt, sizeof h, hipMemcpyDeviceToHost);
            if (rep == 2) std::printf("{\"variant\": \"product\", \"us\": %.1f, \"count\": %u}\n", ms * 1e3, h.n_cand);
        }
    }
    for (int v = 0; v < 4; ++v) {
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(ctr, 0, 8);
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k_find_var, dim3(grid), dim3(256), 0, 0, a, v, ctr);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long h = 0;
            hipMemcpy(&h, ctr, 8, hipMemcpyDeviceToHost);
            if (rep == 2) std::printf("{\"variant\": %d, \"us\": %.1f, \"count\": %llu}\n", v, ms * 1e3, h);
        }
    }
    return 0;
}
