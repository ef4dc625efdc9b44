// Launch entry points of the gfx950 kernels (k_all.hip, k_axis.hip, k_map.hip).
// k_all.hip and k_axis.hip are compiled once per dtype (RDX_T / RDX_TNAME, Makefile) so the
// template-heavy kernels build in parallel; k_dispatch.cpp switches on the runtime dtype.
#pragma once
#include <hip/hip_runtime.h>

#include "rdx_kdesc.h"

#define RDX_KCAT2(a, b) a##_##b
#define RDX_KCAT(a, b) RDX_KCAT2(a, b)
#define RDX_KFN(name) RDX_KCAT(name, RDX_TNAME)

namespace rdx {

hipError_t launch_all_contig(uint32_t dtype, uint32_t op, const KAllContig &a, uint32_t n_chunks, hipStream_t s);
hipError_t launch_all_strided(uint32_t dtype, uint32_t op, const KAllStrided &a, uint32_t n_chunks, hipStream_t s);
hipError_t launch_axis(uint32_t dtype, uint32_t op, const KAxis &a, int cus, hipStream_t s);
hipError_t launch_map(uint32_t dtype, const KMap &a, int cus, hipStream_t s);
hipError_t launch_unshuffle(const uint8_t *in, uint8_t *out, uint64_t len, uint64_t es, int cus, hipStream_t s);
// k_multi.hip: one launch over a heterogeneous batch of all-axes requests
hipError_t launch_multi(const KMultiArgs &m, uint32_t blocks, hipStream_t s);
hipError_t launch_cbor(const KCbor &m, uint32_t blocks, hipStream_t s);
uint64_t cbor_stage_bytes(uint64_t n_tiles);   // the staged form's scratch (k_cbor.hip)
uint32_t cbor_pack_tpg(uint64_t n_tiles);      // ... its tiles per k_cbor_pack workgroup
// k_inflate.hip: gzip / zlib streams (format = rdx_compression), one wavefront per stream
hipError_t launch_inflate(uint32_t format, const uint8_t *const *d_in, const uint64_t *d_in_len, uint64_t n,
                          uint8_t *d_out, uint64_t cap, uint64_t *d_out_len, uint32_t *d_err, hipStream_t s);
hipError_t launch_inflate_table(const uint8_t *const *d_in, const uint64_t *d_in_len, uint8_t *const *d_out_ptrs,
                                const uint64_t *d_caps, const uint32_t *d_n, uint64_t max_n, uint64_t *d_out_len,
                                uint32_t *d_err, hipStream_t s);
// k_blosc2.hip: blosc2 chunks (decode launch, then the filter launch when `filters`)
hipError_t launch_blosc2(const KBlosc2Args &a, bool filters, hipStream_t s);
// after launch_blosc2(a, false) and the zlib-coded streams' inflate (launch_inflate_table): fold their
// results into the chunks' errors, then the filter launch
hipError_t launch_blosc2_zcheck(const KBlosc2Args &a, hipStream_t s);
// after launch_blosc2(a, false): the zstd-coded streams of the table (rows [z_capacity, 2 z_capacity))
hipError_t launch_blosc2_zstd(const KBlosc2Args &a, hipStream_t s);

#define RDX_DECLARE_DTYPE(tn)                                                                                  \
    hipError_t launch_all_contig_##tn(uint32_t op, const KAllContig &a, uint32_t n_chunks, hipStream_t s);    \
    hipError_t launch_all_strided_##tn(uint32_t op, const KAllStrided &a, uint32_t n_chunks, hipStream_t s);  \
    hipError_t launch_axis_##tn(uint32_t op, const KAxis &a, int cus, hipStream_t s);
RDX_DECLARE_DTYPE(i32)
RDX_DECLARE_DTYPE(i64)
RDX_DECLARE_DTYPE(u32)
RDX_DECLARE_DTYPE(u64)
RDX_DECLARE_DTYPE(f32)
RDX_DECLARE_DTYPE(f64)
#undef RDX_DECLARE_DTYPE

}  // namespace rdx
