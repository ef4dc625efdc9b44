// Probe (tuning only): k_pinf_find on one zlib stream read from a file, timed with HIP events.
//   hipcc -O3 --offload-arch=gfx950 -I reductionist-rs_amd/csrc tools/probe_pinf_find.hip -o tools/probe_pinf_find
//   tools/probe_pinf_find stream.zlib
// (the product kernel: its time, candidates and screen survivors)
#include "../reductionist-rs_amd/csrc/k_pinflate.hip"

#include <cstdio>
#include <vector>

using namespace rdx;

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
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
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
            if (rep == 2)
                std::printf("{\"variant\": \"product\", \"us\": %.1f, \"count\": %u, \"survivors\": %u}\n", ms * 1e3,
                            h.n_cand, h.n_surv);
        }
    }
    return 0;
}
