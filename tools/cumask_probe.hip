// Does a CU-masked stream (hipExtStreamCreateWithCUMask) keep its mask (a) eagerly, (b) for a
// kernel captured into a HIP graph from that stream and replayed on it, (c) replayed on
// another stream? Each block records which CU it ran on (__smid: XCC, SE, CU); the probe
// prints how many distinct CUs each launch touched. VERDICT r05 item 2 asked for this check
// before a masked weight-gradient stream is worth building into the step graph.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/cumask_probe.hip -o tools/bin/cumask_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ __launch_bounds__(256) void where_kernel(unsigned* out, float* sink, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  for (int i = 0; i < iters; ++i) a = a * b + 1e-7f;  // keep the block resident a while
  if (threadIdx.x == 0) out[blockIdx.x] = __smid();
  if (a == -1.f) sink[threadIdx.x] = a;  // never true; keeps the loop
}

static int distinct(const std::vector<unsigned>& v) {
  return (int)std::set<unsigned>(v.begin(), v.end()).size();
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  printf("device %s, %d CUs\n", prop.gcnArchName, ncu);
  const int blocks = 8192, iters = 20000;
  unsigned* d_out;
  float* sink;
  CK(hipMalloc(&d_out, blocks * sizeof(unsigned)));
  CK(hipMalloc(&sink, 256 * sizeof(float)));
  std::vector<unsigned> h(blocks);

  const int nwords = (ncu + 31) / 32;
  std::vector<uint32_t> mask(nwords, 0u);
  const int keep = ncu / 4;  // a quarter of the CUs, the lowest-numbered
  for (int c = 0; c < keep; ++c) mask[c / 32] |= 1u << (c % 32);
  hipStream_t plain, masked;
  CK(hipStreamCreate(&plain));
  CK(hipExtStreamCreateWithCUMask(&masked, nwords, mask.data()));
  std::vector<uint32_t> got(nwords, 0u);
  CK(hipExtStreamGetCUMask(masked, nwords, got.data()));
  int bits = 0;
  for (uint32_t w : got) bits += __builtin_popcount(w);
  printf("masked stream: %d of %d CUs in its mask\n", bits, ncu);

  bool verbose = false;
  auto run = [&](const char* name, auto launch) -> int {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipMemset(d_out, 0xff, blocks * sizeof(unsigned)));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, plain));
    if (launch()) return 1;
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(b, plain));
    CK(hipEventSynchronize(b));
    CK(hipMemcpy(h.data(), d_out, blocks * sizeof(unsigned), hipMemcpyDeviceToHost));
    printf("%-44s distinct CUs %4d\n", name, distinct(h));
    if (verbose) {  // the ids (__smid: XCC << (SE bits + CU bits) | SE << CU bits | CU)
      std::set<unsigned> ids(h.begin(), h.end());
      for (unsigned id : ids) printf(" %x", id);
      printf("\n");
    }
    return 0;
  };

  if (run("eager, plain stream", [&] {
        where_kernel<<<blocks, 256, 0, plain>>>(d_out, sink, iters);
        return hipGetLastError() != hipSuccess;
      }))
    return 1;
  verbose = true;
  if (run("eager, masked stream", [&] {
        where_kernel<<<blocks, 256, 0, masked>>>(d_out, sink, iters);
        return hipGetLastError() != hipSuccess;
      }))
    return 1;

  verbose = false;
  hipGraph_t graph;
  hipGraphExec_t exec;
  CK(hipStreamBeginCapture(masked, hipStreamCaptureModeGlobal));
  where_kernel<<<blocks, 256, 0, masked>>>(d_out, sink, iters);
  CK(hipStreamEndCapture(masked, &graph));
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  if (run("graph captured on masked, replayed on masked", [&] {
        return hipGraphLaunch(exec, masked) != hipSuccess;
      }))
    return 1;
  if (run("graph captured on masked, replayed on plain", [&] {
        return hipGraphLaunch(exec, plain) != hipSuccess;
      }))
    return 1;

  // a two-branch graph: the masked stream forked from a plain capture (the step graph's shape)
  hipGraph_t g2;
  hipGraphExec_t e2;
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipStreamBeginCapture(plain, hipStreamCaptureModeGlobal));
  CK(hipEventRecord(fork, plain));
  CK(hipStreamWaitEvent(masked, fork, 0));
  where_kernel<<<blocks, 256, 0, masked>>>(d_out, sink, iters);
  CK(hipEventRecord(join, masked));
  CK(hipStreamWaitEvent(plain, join, 0));
  CK(hipStreamEndCapture(plain, &g2));
  CK(hipGraphInstantiate(&e2, g2, nullptr, nullptr, 0));
  if (run("forked branch on masked, graph on plain", [&] {
        return hipGraphLaunch(e2, plain) != hipSuccess;
      }))
    return 1;
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphExecDestroy(e2));
  CK(hipGraphDestroy(graph));
  CK(hipGraphDestroy(g2));
  CK(hipStreamDestroy(masked));
  CK(hipStreamDestroy(plain));
  return 0;
}
