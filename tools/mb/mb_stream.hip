// mb_stream.hip -- microbenchmarks of the C3 SpMV access pattern (tools only,
// not part of the product).  Buffers have C3's sizes and 64-row block layout
// (7-pt Laplacian 216^3: blk_k from the real row_ptr).  Each variant reads the
// val/col windows of every 64-row block and varies ONE thing:
//   1 vgpr    : val/col window -> VGPRs (16 B/lane), one wave per block
//   2 vgpr+ry : 1 + row_ptr loads + y store (512 B per block)
//   3 dma     : window -> LDS by global_load_lds_dwordx4, one wave per block
//   4 dma+ry  : 3 + row_ptr + y
//   5 exact   : 2 but loads only the 16 B pieces the block needs (exec mask)
//   6 persist : 2 as persistent waves (grid = 8 x CUs x 4 waves), loop
//   7 copy    : float4 copy of val (read 562 MB, write 562 MB) -- reference
// Build: hipcc --offload-arch=gfx950 -O3 -o mb_stream mb_stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef __attribute__((address_space(3))) void lds_void;

struct Args {
  const double *val; const int *col; const int *rp; const int *blk_k; const int *blk_row;
  double *y; double *sink; int nblk;
};

template <int MODE>
__global__ __launch_bounds__(256) void k_mb(Args a) {
  __shared__ __attribute__((aligned(16))) char lds[4][6144];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int nwaves = gridDim.x * 4;
  int b = blockIdx.x * 4 + wid;
  double acc = 0;
  for (; b < a.nblk; b += (MODE == 6 ? nwaves : a.nblk)) {
    const int k0 = a.blk_k[b], k1 = a.blk_k[b + 1];
    const int kb = k0 & ~3;
    if (MODE == 1 || MODE == 2 || MODE == 6 || MODE >= 9) {  // (12, 13 too)
      const double4 *vv = (const double4 *)(a.val + kb);  // 32 B/lane x 2 = 4 KB
      const int4 *cc = (const int4 *)(a.col + kb);
      double2 v0 = ((const double2 *)(a.val + kb))[lane];
      double2 v1 = ((const double2 *)(a.val + kb))[lane + 64];
      double2 v2 = ((const double2 *)(a.val + kb))[lane + 128];
      double2 v3 = ((const double2 *)(a.val + kb))[lane + 192];
      int4 c0 = cc[lane], c1 = cc[lane + 64];
      (void)vv;
      acc += v0.x + v1.y + v2.x + v3.y + (double)(c0.x + c1.w);
    } else if (MODE == 5) {
      const int m = k1 - kb;  // elements needed
      double2 v[4] = {}; int4 c[2] = {};
#pragma unroll
      for (int q = 0; q < 4; ++q) if ((q * 64 + lane) * 2 < m) v[q] = ((const double2 *)(a.val + kb))[q * 64 + lane];
#pragma unroll
      for (int q = 0; q < 2; ++q) if ((q * 64 + lane) * 4 < m) c[q] = ((const int4 *)(a.col + kb))[q * 64 + lane];
      acc += v[0].x + v[1].y + v[2].x + v[3].y + (double)(c[0].x + c[1].w);
    } else if (MODE == 3 || MODE == 4) {
      char *L = lds[wid];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds((const void *)(a.val + kb + q * 128 + lane * 2), (lds_void *)(L + q * 1024), 16, 0, 0);
#pragma unroll
      for (int q = 0; q < 2; ++q)
        __builtin_amdgcn_global_load_lds((const void *)(a.col + kb + q * 256 + lane * 4), (lds_void *)(L + 4096 + q * 1024), 16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0x0F70);
      acc += ((double *)L)[lane * 7 % 512] + ((int *)(L + 4096))[lane];
    }
    if (MODE == 9) {  // y store only
      const int r0 = a.blk_row[b], nr = a.blk_row[b + 1] - r0;
      if (lane < nr) a.y[r0 + lane] = acc;
    }
    if (MODE == 10) {  // row_ptr only
      const int r0 = a.blk_row[b], nr = a.blk_row[b + 1] - r0;
      if (lane < nr) acc += (double)(a.rp[r0 + lane + 1] - a.rp[r0 + lane]);
    }
    if (MODE == 11) {  // row_ptr + nt y store
      const int r0 = a.blk_row[b], nr = a.blk_row[b + 1] - r0;
      if (lane < nr) {
        const int j0 = a.rp[r0 + lane], j1 = a.rp[r0 + lane + 1];
        __builtin_nontemporal_store(acc + (double)(j1 - j0), a.y + r0 + lane);
      }
    }
    if (MODE == 13) {  // row_ptr + y as 16 B per lane from half the lanes
      const int r0 = a.blk_row[b], nr = a.blk_row[b + 1] - r0;
      double v = 0;
      if (lane < nr) {
        const int j0 = a.rp[r0 + lane], j1 = a.rp[r0 + lane + 1];
        v = acc + (double)(j1 - j0);
      }
      const double w = __shfl_down(v, 1);
      if ((lane & 1) == 0 && lane + 1 < nr)
        *(double2 *)(a.y + r0 + lane) = make_double2(v, w);
      else if ((lane & 1) == 0 && lane < nr)
        a.y[r0 + lane] = v;
    }
    if (MODE == 2 || MODE == 4 || MODE == 5 || MODE == 6) {
      const int r0 = a.blk_row[b], nr = a.blk_row[b + 1] - r0;
      if (lane < nr) {
        const int j0 = a.rp[r0 + lane], j1 = a.rp[r0 + lane + 1];
        a.y[r0 + lane] = acc + (double)(j1 - j0);
      }
    }
  }
  if (MODE == 1 || MODE == 3 || MODE == 10) if (acc == 12345.678) a.sink[0] = acc;
}

// mode 12: stream + row_ptr per wave; y staged in LDS and written by the
// whole workgroup as one contiguous 256-row (2 KiB) burst after a barrier
__global__ __launch_bounds__(256) void k_mb12(Args a) {
  __shared__ double ys[256];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b = blockIdx.x * 4 + wid;
  double acc = 0;
  if (b < a.nblk) {
    const int k0 = a.blk_k[b];
    const int kb = k0 & ~3;
    double2 v0 = ((const double2 *)(a.val + kb))[lane];
    double2 v1 = ((const double2 *)(a.val + kb))[lane + 64];
    double2 v2 = ((const double2 *)(a.val + kb))[lane + 128];
    double2 v3 = ((const double2 *)(a.val + kb))[lane + 192];
    const int4 *cc = (const int4 *)(a.col + kb);
    int4 c0 = cc[lane], c1 = cc[lane + 64];
    acc += v0.x + v1.y + v2.x + v3.y + (double)(c0.x + c1.w);
    const int r0 = a.blk_row[b], nr = a.blk_row[b + 1] - r0;
    if (lane < nr) acc += (double)(a.rp[r0 + lane + 1] - a.rp[r0 + lane]);
  }
  ys[threadIdx.x] = acc;
  __syncthreads();
  const int row = blockIdx.x * 256 + threadIdx.x;  // 64-row blocks: contiguous rows
  if (row < a.nblk * 64 && row < (int)(a.nblk) * 64) a.y[row] = ys[threadIdx.x];
}

__global__ void k_copy(const double2 *__restrict__ s, double2 *__restrict__ d, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}
__global__ void k_read(const double2 *__restrict__ s, double *sink, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  double acc = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) { double2 v = s[i]; acc += v.x + v.y; }
  if (acc == 12345.678) sink[0] = acc;
}

int main() {
  const int N = 216, n = N * N * N;
  std::vector<int> rp(n + 1); rp[0] = 0;
  for (int i = 0; i < n; ++i) {
    int x = i % N, y = (i / N) % N, z = i / (N * N);
    int c = 1 + (x > 0) + (x < N - 1) + (y > 0) + (y < N - 1) + (z > 0) + (z < N - 1);
    rp[i + 1] = rp[i] + c;
  }
  const int nnz = rp[n];
  const int nblk = (n + 63) / 64;
  std::vector<int> bk(nblk + 1), br(nblk + 1);
  for (int b = 0; b <= nblk; ++b) { br[b] = std::min(n, b * 64); bk[b] = rp[br[b]]; }
  double *val, *y, *sink, *dst; int *col, *drp, *dbk, *dbr;
  const size_t pad = 4096;
  CK(hipMalloc(&val, (nnz + pad) * 8)); CK(hipMalloc(&col, (nnz + pad) * 4));
  CK(hipMalloc(&drp, (n + 1) * 4)); CK(hipMalloc(&dbk, (nblk + 1) * 4)); CK(hipMalloc(&dbr, (nblk + 1) * 4));
  CK(hipMalloc(&y, (size_t)n * 8)); CK(hipMalloc(&sink, 64)); CK(hipMalloc(&dst, (nnz + pad) * 8));
  CK(hipMemset(val, 0, (nnz + pad) * 8)); CK(hipMemset(col, 0, (nnz + pad) * 4));
  CK(hipMemcpy(drp, rp.data(), (n + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbk, bk.data(), (nblk + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbr, br.data(), (nblk + 1) * 4, hipMemcpyHostToDevice));
  Args a{val, col, drp, dbk, dbr, y, sink, nblk};
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const double stream = (double)nnz * 12, ry = (double)n * 4 + (double)n * 8;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char *name, auto launch, double bytes) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    float best = 1e9, tot = 0; const int R = 20;
    for (int r = 0; r < R; ++r) {
      CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms); tot += ms;
    }
    printf("%-34s avg %8.2f us  min %8.2f us  %7.1f GB/s (of %6.1f MB)\n", name, 1e3 * tot / R, 1e3 * best,
           bytes / (tot / R * 1e-3) / 1e9, bytes / 1e6);
  };
  const int g1 = (nblk + 3) / 4;
  run("1 vgpr window", [&] { hipLaunchKernelGGL(k_mb<1>, dim3(g1), dim3(256), 0, 0, a); }, stream);
  run("2 vgpr window + rp + y", [&] { hipLaunchKernelGGL(k_mb<2>, dim3(g1), dim3(256), 0, 0, a); }, stream + ry);
  run("3 dma window", [&] { hipLaunchKernelGGL(k_mb<3>, dim3(g1), dim3(256), 0, 0, a); }, stream);
  run("4 dma window + rp + y", [&] { hipLaunchKernelGGL(k_mb<4>, dim3(g1), dim3(256), 0, 0, a); }, stream + ry);
  run("5 exact pieces + rp + y", [&] { hipLaunchKernelGGL(k_mb<5>, dim3(g1), dim3(256), 0, 0, a); }, stream + ry);
  run("9 vgpr window + y", [&] { hipLaunchKernelGGL(k_mb<9>, dim3(g1), dim3(256), 0, 0, a); }, stream + (double)n * 8);
  run("10 vgpr window + rp", [&] { hipLaunchKernelGGL(k_mb<10>, dim3(g1), dim3(256), 0, 0, a); }, stream + (double)n * 4);
  run("11 vgpr window + rp + nt y", [&] { hipLaunchKernelGGL(k_mb<11>, dim3(g1), dim3(256), 0, 0, a); }, stream + ry);
  run("12 vgpr window + rp + y (WG 2 KiB burst)", [&] { hipLaunchKernelGGL(k_mb12, dim3(g1), dim3(256), 0, 0, a); }, stream + ry);
  run("13 vgpr window + rp + y (16 B/lane)", [&] { hipLaunchKernelGGL(k_mb<13>, dim3(g1), dim3(256), 0, 0, a); }, stream + ry);
  run("1 vgpr window (again)", [&] { hipLaunchKernelGGL(k_mb<1>, dim3(g1), dim3(256), 0, 0, a); }, stream);
  run("2 vgpr window + rp + y (again)", [&] { hipLaunchKernelGGL(k_mb<2>, dim3(g1), dim3(256), 0, 0, a); }, stream + ry);
  for (int m : {4})
  { char nm[64]; snprintf(nm, 64, "6 persistent x%d + rp + y", m);
    run(nm, [&] { hipLaunchKernelGGL(k_mb<6>, dim3(cus * m), dim3(256), 0, 0, a); }, stream + ry); }
  const size_t n2 = (size_t)nnz / 2;
  run("7 float4 copy of val", [&] { hipLaunchKernelGGL(k_copy, dim3(cus * 16), dim3(256), 0, 0, (const double2 *)val, (double2 *)dst, n2); }, 2.0 * n2 * 16);
  run("8 float4 read of val", [&] { hipLaunchKernelGGL(k_read, dim3(cus * 16), dim3(256), 0, 0, (const double2 *)val, sink, n2); }, 1.0 * n2 * 16);
  run("8b float4 read of val (grid 64x)", [&] { hipLaunchKernelGGL(k_read, dim3(cus * 64), dim3(256), 0, 0, (const double2 *)val, sink, n2); }, 1.0 * n2 * 16);
  printf("nnz %d nblk %d cus %d\n", nnz, nblk, cus);
  return 0;
}
