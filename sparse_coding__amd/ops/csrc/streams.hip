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

// Upload an instantiated graph to the device ahead of its first launch.  Without it the first
// hipGraphLaunch of a freshly captured multi-step graph pays the upload inline (on MI355X several
// hundred microseconds for a 40-60 node graph), which lands inside whatever region times it.
int sc_graph_upload(void* exec, void* stream) {
  if (hipGraphUpload(reinterpret_cast<hipGraphExec_t>(exec), reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
    return 3;
  return 0;
}

}  // extern "C"
