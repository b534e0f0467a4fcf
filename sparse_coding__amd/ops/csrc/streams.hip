// HIP streams restricted to a subset of compute units (hipExtStreamCreateWithCUMask), for
// running a memory-bound kernel (the streaming Adam) beside MFMA-bound GEMMs on disjoint CUs
// instead of letting both grids compete for every CU.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

extern "C" {

// mask: nwords 32-bit words, bit i = compute unit i.  Returns the stream in *out.
int sc_stream_create_cumask(const uint32_t* mask, int nwords, void** out) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask) != hipSuccess) return 3;
  *out = reinterpret_cast<void*>(s);
  return 0;
}

int sc_stream_destroy(void* s) {
  return hipStreamDestroy(reinterpret_cast<hipStream_t>(s)) == hipSuccess ? 0 : 3;
}

}  // extern "C"
