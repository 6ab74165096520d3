// graph_ring_repro.hip — no mfea code: a captured hipGraph of `nodes` trivial
// kernel nodes (the engine's chunk graphs hold 57: 8 iterations × 7 kernels +
// k_cg_advance) replayed `launches` times, to run under
//   rocprofv3 --kernel-trace --stats -- ./graph_ring_repro [nodes] [launches]
// without DEBUG_CLR_GRAPH_PACKET_CAPTURE=0.  The engine's rocprofv3 SIGSEGV
//  faulted one byte past a 1 MiB HSA queue ring inside the
// tracer's queue interception of a graph launch; if this program faults the
// same way, the fault needs nothing of the engine's.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_touch(float* p, int i) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[i] = p[i] + 1.0f;
}

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                                    \
    }                                                              \
  } while (0)

int main(int argc, char** argv) {
  const int nodes = argc > 1 ? std::atoi(argv[1]) : 57;
  const int launches = argc > 2 ? std::atoi(argv[2]) : 20000;
  float* p = nullptr;
  CK(hipMalloc(&p, sizeof(float) * 1024));
  CK(hipMemset(p, 0, sizeof(float) * 1024));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < nodes; ++k) hipLaunchKernelGGL(k_touch, dim3(64), dim3(64), 0, s, p, k % 1024);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int r = 0; r < launches; ++r) {
    CK(hipGraphLaunch(ge, s));
    if ((r & 1023) == 1023) CK(hipStreamSynchronize(s));
  }
  CK(hipStreamSynchronize(s));
  float h0 = 0;
  CK(hipMemcpy(&h0, p, sizeof(float), hipMemcpyDeviceToHost));
  std::printf("{\"nodes\": %d, \"launches\": %d, \"p0\": %.0f}\n", nodes, launches, h0);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(p));
  return 0;
}
