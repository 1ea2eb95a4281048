// fec_status.h -- where a HIP runtime call failed: FEC_HIP(call) returns FEC_ERR_HIP from the
// enclosing function after recording the call's error name and source line, which the C ABI
// reports through fec_last_error (include/fec_amd.h) and the Python layer appends to FecError.
#pragma once

#include <hip/hip_runtime.h>

namespace fec {
int hip_failed(hipError_t e, const char* site);  // records, returns FEC_ERR_HIP
}

#define FEC_STR2_(x) #x
#define FEC_STR_(x) FEC_STR2_(x)
#define FEC_HIP(call)                                                                              \
    do {                                                                                           \
        const hipError_t fec_e_ = (call);                                                          \
        if (fec_e_ != hipSuccess) return ::fec::hip_failed(fec_e_, __FILE__ ":" FEC_STR_(__LINE__) ": " #call); \
    } while (0)
