// Host-side planning for one request: the checks operation<T>() runs before touching data
// (src/app.rs:163-183, src/array.rs:18-63, src/filters/shuffle.rs:21), the numpy->ndarray
// hyperslab translation (src/array.rs:93-144) and its canonicalisation into one of four kernel
// shapes.  Pure C++ (no HIP): also backs rdx_plan()/rdx_validate_request() on CPU-only hosts.
#pragma once
#include <vector>

#include "../../include/rdx.h"
#include "rdx_kdesc.h"

namespace rdx {

enum class Mode { AllContig, AllStrided, Axis, Map };

struct ExecPlan {
    rdx_response_info info{};
    uint32_t op = 0, dtype = 0, esz = 0;
    bool is_float = false;
    bool need_rank = false;            // float min/max: ±0 tie rule needs the fold order rank
    uint64_t chunk_elems = 0;          // chunk_len / sizeof(T)
    std::vector<uint64_t> unfused_es;  // unshuffle passes into scratch, in APPLICATION order
    bool fused = false;                // last decode (filters[0]) fused into the op kernel
    bool bswap = false;
    KMissing miss{};                   // list pointer filled at launch
    std::vector<uint64_t> miss_list;   // sorted list for long missing_values
    Mode mode = Mode::AllContig;
    KAllContig all_contig{};
    KAllStrided all_strided{};
    KAxis axis{};
    KMap map{};
};

// Full structural validation of a request (src/models.rs:179-313) with typed missing values.
rdx_status validate_request(const rdx_request &req);
// Everything needed to launch; returns the first error operation<T>() would raise.
rdx_status make_plan(const rdx_request &req, uint64_t chunk_len, ExecPlan &plan);

uint32_t dtype_size(uint32_t dtype);
// RDX_E_UNSUPPORTED with its rdx_unsupported_reason recorded for this thread (rdx_last_unsupported_reason).
rdx_status unsupported(uint32_t reason);
uint32_t last_unsupported();
Div make_div(uint32_t d);

}  // namespace rdx
