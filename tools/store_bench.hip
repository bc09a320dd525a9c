// Per-CU global-store throughput by store-instruction shape: one 8-wave workgroup per
// CU (96 KiB of LDS claimed) writes 128-KiB tiles (128 rows x 1 KiB, row pitch `ld`)
// with 16-B-per-lane stores whose 64 lanes cover R rows x (1024 / R) contiguous bytes
// each (R = 16 is the GEMM epilogue's shape: 16 rows x 64 B). Prints, per R and grid,
// the median / p90 per-wave issue and drain cycles (s_memtime) and the kernel rate.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/store_bench.hip -o tools/_store_bench
//   ./tools/_store_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                            \
  do {                                                                   \
    if ((x) != hipSuccess) {                                             \
      std::fprintf(stderr, "%s failed at line %d\n", #x, __LINE__);      \
      return 1;                                                          \
    }                                                                    \
  } while (0)

constexpr int kTileBytes = 128 * 1024, kReps = 4;

template <int R>
__global__ __launch_bounds__(512) void store_kernel(char* out, int ld, unsigned long long* stamps) {
  extern __shared__ char smem[];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  constexpr int lpr = 64 / R, chunk = 1024 / R, groups = 128 / R;
  const int r_in = lane / lpr, c_in = lane % lpr;
  uint4 v = {(unsigned)t, (unsigned)blockIdx.x, 1u, 2u};
  if (t == 0) smem[0] = 1;  // the LDS claim is real
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), issue = 0, drain = 0;
  for (int rep = 0; rep < kReps; ++rep) {
    char* base = out + ((size_t)rep * gridDim.x + blockIdx.x) * 128 * (size_t)ld;
    const unsigned long long a = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int s = w * 16 + k;
      const int rg = s % groups, cc = s / groups;
      *(uint4*)(base + (size_t)(rg * R + r_in) * ld + cc * chunk + c_in * 16) = v;
      v.z += 1u;
    }
    const unsigned long long b = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    issue += b - a;
    drain += c - b;
    __syncthreads();
  }
  (void)t0;
  if (lane == 0) {
    stamps[(blockIdx.x * 8 + w) * 2] = issue / kReps;
    stamps[(blockIdx.x * 8 + w) * 2 + 1] = drain / kReps;
  }
}

template <int R>
int run(char* out, int ld, unsigned long long* st, int grid) {
  auto k = store_kernel<R>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) k<<<grid, 512, 96 * 1024>>>(out, ld, st);
  CK(hipEventRecord(e0));
  const int n = 20;
  for (int i = 0; i < n; ++i) k<<<grid, 512, 96 * 1024>>>(out, ld, st);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(grid * 16);
  CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<unsigned long long> is, dr;
  for (int i = 0; i < grid * 8; ++i) {
    is.push_back(h[2 * i]);
    dr.push_back(h[2 * i + 1]);
  }
  std::sort(is.begin(), is.end());
  std::sort(dr.begin(), dr.end());
  const double us = ms * 1e3 / n;
  const double bytes = (double)grid * kTileBytes * kReps;
  std::printf("R=%2d (%4d B per row) grid=%4d: issue med %6llu p90 %6llu cyc, drain med %6llu p90 %6llu cyc per "
              "128 KiB tile; kernel %7.1f us = %6.0f GB/s, %5.1f B/cyc/CU at 2.2 GHz\n",
              R, 1024 / R, grid, is[is.size() / 2], is[is.size() * 9 / 10], dr[dr.size() / 2],
              dr[dr.size() * 9 / 10], us, bytes / us / 1e3, bytes / grid / (us * 2200.0));
  return 0;
}

int main() {
  const int ld = 6144;  // the QKV output row pitch (3072 bf16)
  char* out;
  unsigned long long* st;
  CK(hipMalloc(&out, (size_t)kReps * 256 * 128 * ld + 4096));
  CK(hipMalloc(&st, 256 * 16 * 8));
  for (int grid : {32, 256}) {
    if (run<16>(out, ld, st, grid) || run<8>(out, ld, st, grid) || run<4>(out, ld, st, grid) ||
        run<2>(out, ld, st, grid) || run<1>(out, ld, st, grid))
      return 1;
  }
  CK(hipFree(out));
  CK(hipFree(st));
  return 0;
}
