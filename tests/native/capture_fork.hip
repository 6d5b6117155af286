// capture_fork.hip -- the partitioned solver's per-iteration stream shape
// (csrc/cgx_dist.cpp phase_pack / phase_halo / phase_spmv), captured as a
// hipGraph and replayed, against the same work run eagerly:
//   st:      record ev_fork                        (fork)
//   st_comm: wait ev_fork; pack kernel; D2D copy into the ghost tail
//            (stands in for ncclSend/Recv); record ev_halo
//   st:      interior kernel || the above; wait ev_halo (join);
//            boundary kernel; update kernel
// Round 2 saw a host crash capturing a variant of this shape whose forked
// stream held only event records and a wait on its own event; this program
// checks the shape libcgx uses now: 16 iterations per graph, replayed 4
// times, bit-identical to eager.  Exit 0 = pass.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,            \
              hipGetErrorString(e_));                                      \
      return 2;                                                            \
    }                                                                      \
  } while (0)

constexpr int N = 1 << 20, G = 4096;  // rows, ghost / send rows

__global__ void k_pack(const double *x, const int *idx, double *buf) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < G) buf[i] = x[idx[i]] * 0.5 + 1.0;
}
__global__ void k_interior(const double *x, double *y) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256)
    y[i] = 0.25 * x[i] + (i > 0 ? 0.125 * x[i - 1] : 0.0);
}
__global__ void k_boundary(const double *ghost, double *y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < G) y[N - G + i] += 0.5 * ghost[i];
}
__global__ void k_update(double *x, const double *y) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256)
    x[i] = y[i] + 0.75 * x[i];
}

struct Ctx {
  hipStream_t st, st_comm;
  hipEvent_t ev_fork, ev_halo;
  double *x, *y, *ghost, *buf;
  int *idx;
};

static int iteration(Ctx &c) {
  CK(hipEventRecord(c.ev_fork, c.st));
  CK(hipStreamWaitEvent(c.st_comm, c.ev_fork, 0));
  hipLaunchKernelGGL(k_pack, dim3(G / 256), dim3(256), 0, c.st_comm, c.x, c.idx, c.buf);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(c.ghost, c.buf, G * 8, hipMemcpyDeviceToDevice, c.st_comm));
  CK(hipEventRecord(c.ev_halo, c.st_comm));
  hipLaunchKernelGGL(k_interior, dim3(1024), dim3(256), 0, c.st, c.x, c.y);
  CK(hipGetLastError());
  CK(hipStreamWaitEvent(c.st, c.ev_halo, 0));
  hipLaunchKernelGGL(k_boundary, dim3(G / 256), dim3(256), 0, c.st, c.ghost, c.y);
  hipLaunchKernelGGL(k_update, dim3(1024), dim3(256), 0, c.st, c.x, c.y);
  CK(hipGetLastError());
  return 0;
}

static int reset(Ctx &c) {
  std::vector<double> h(N);
  for (int i = 0; i < N; ++i) h[i] = (double)((i * 2654435761u) % 1000) / 997.0;
  CK(hipMemcpy(c.x, h.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemset(c.y, 0, N * 8));
  CK(hipMemset(c.ghost, 0, G * 8));
  return 0;
}

int main() {
  Ctx c;
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  CK(hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&c.st_comm, hipStreamNonBlocking, greatest));
  CK(hipEventCreateWithFlags(&c.ev_fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&c.ev_halo, hipEventDisableTiming));
  CK(hipMalloc((void **)&c.x, N * 8));
  CK(hipMalloc((void **)&c.y, N * 8));
  CK(hipMalloc((void **)&c.ghost, G * 8));
  CK(hipMalloc((void **)&c.buf, G * 8));
  CK(hipMalloc((void **)&c.idx, G * 4));
  std::vector<int> idx(G);
  for (int i = 0; i < G; ++i) idx[i] = (i * 7919) % N;
  CK(hipMemcpy(c.idx, idx.data(), G * 4, hipMemcpyHostToDevice));

  const int iters = 64, batch = 16;
  // eager
  if (reset(c)) return 2;
  for (int i = 0; i < iters; ++i)
    if (iteration(c)) return 2;
  CK(hipStreamSynchronize(c.st));
  std::vector<double> ref(N), got(N);
  CK(hipMemcpy(ref.data(), c.x, N * 8, hipMemcpyDeviceToHost));
  // captured: `batch` iterations per graph, replayed
  if (reset(c)) return 2;
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  CK(hipStreamBeginCapture(c.st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < batch; ++i)
    if (iteration(c)) return 2;
  CK(hipStreamEndCapture(c.st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < iters / batch; ++i) CK(hipGraphLaunch(ge, c.st));
  CK(hipStreamSynchronize(c.st));
  CK(hipMemcpy(got.data(), c.x, N * 8, hipMemcpyDeviceToHost));
  const bool same = memcmp(ref.data(), got.data(), N * 8) == 0;
  printf("capture_fork: %d iterations, graph of %d, %s\n", iters, batch,
         same ? "bit-identical to eager" : "MISMATCH");
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return same ? 0 : 1;
}
