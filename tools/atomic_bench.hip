// Per-CU throughput of the residual-add forms a GEMM epilogue can use on an fp32 tile
// (128 rows x 256 fp32 columns = 128 KiB at row pitches from 4 KiB -- the out-proj / c_proj
// output -- up), one 8-wave workgroup per CU (96 KiB of LDS claimed):
//   store   16-B stores only (no residual: the floor)
//   rmw     16-B load + add + 16-B store (the shipped epilogue: x += v in registers)
//   atom4   four dword float atomic adds per 16-B lane chunk (the MFMA lane layout as is)
//   atomrow dword float atomic adds, 16 lanes per 64-B row segment (a transposed layout)
//   storeq / rmwq  store / rmw with the lanes re-ordered: the 4 lanes of a quad cover one
//                  row's 64 B (the same addresses per instruction as store / rmw, whose
//                  consecutive lanes are consecutive rows -- the MFMA accumulator layout)
// Per form and grid: median / p90 per-wave issue and drain cycles (s_memtime) and the
// kernel rate. Every launch adds 1 to each tile element (store: writes 1), and the bench
// checks the final values against the count of launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics tools/atomic_bench.hip -o tools/_atomic_bench
//   ./tools/_atomic_bench
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

constexpr int kRows = 128, kReps = 4;
__constant__ int kLd;  // row pitch in floats (set per run)
static int hLd = 1024;
enum Form { STORE = 0, RMW = 1, ATOM4 = 2, ATOMROW = 3, STOREQ = 4, RMWQ = 5 };

template <int F>
__global__ __launch_bounds__(512) void epi_kernel(float* out, unsigned long long* stamps) {
  extern __shared__ char smem[];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, fr = lane & 15, fq = lane >> 4;
  if (t == 0) smem[0] = 1;  // the LDS claim is real
  unsigned long long issue = 0, drain = 0;
  const float4 v = {1.f, 1.f, 1.f, 1.f};
  for (int rep = 0; rep < kReps; ++rep) {
    float* base = out + ((size_t)rep * gridDim.x + blockIdx.x) * kRows * (size_t)kLd;
    const unsigned long long a = __builtin_amdgcn_s_memtime();
    if constexpr (F == ATOMROW) {
      // 64 instructions per wave, each 4 rows x 64 B (16 lanes per row segment)
#pragma unroll 8
      for (int k = 0; k < 64; ++k) {
        const int s = w * 64 + k, rg = s % 32, cc = s / 32;
        unsafeAtomicAdd(base + (size_t)(rg * 4 + fq) * kLd + cc * 16 + fr, 1.f);
      }
    } else {
      // 16 blocks per wave, each 16 rows x 64 B (lane: row fr, 16 B at column group fq)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int s = w * 16 + k, rg = s % 8, cc = s / 8;
        const int row = (F == STOREQ || F == RMWQ) ? lane >> 2 : fr, col = (F == STOREQ || F == RMWQ) ? lane & 3 : fq;
        float* p = base + (size_t)(rg * 16 + row) * kLd + cc * 16 + 4 * col;
        if constexpr (F == STORE || F == STOREQ) {
          *(float4*)p = v;
        } else if constexpr (F == RMW || F == RMWQ) {
          float4 r = *(const float4*)p;
          r.x += 1.f;
          r.y += 1.f;
          r.z += 1.f;
          r.w += 1.f;
          *(float4*)p = r;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) unsafeAtomicAdd(p + e, 1.f);
        }
      }
    }
    const unsigned long long b = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    issue += b - a;
    drain += c - b;
    __syncthreads();
  }
  if (lane == 0) {
    stamps[(blockIdx.x * 8 + w) * 2] = issue / kReps;
    stamps[(blockIdx.x * 8 + w) * 2 + 1] = drain / kReps;
  }
}

template <int F>
int run(const char* name, float* out, unsigned long long* st, int grid) {
  auto k = epi_kernel<F>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(kLd), &hLd, sizeof(int)));
  const size_t n = (size_t)kReps * grid * kRows * hLd;
  CK(hipMemset(out, 0, n * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int warm = 3, iters = 20;
  for (int i = 0; i < warm; ++i) k<<<grid, 512, 96 * 1024>>>(out, st);
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) k<<<grid, 512, 96 * 1024>>>(out, st);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  // check: the 256 columns of every tile row got warm + iters adds (store: 1.0)
  std::vector<float> h(n);
  CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
  const float want = (F == STORE || F == STOREQ) ? 1.f : (float)(warm + iters);
  size_t bad = 0;
  for (size_t r = 0; r < n / hLd; ++r)
    for (int c = 0; c < 256; ++c) bad += h[r * hLd + c] != want;
  std::vector<unsigned long long> hs(grid * 16);
  CK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
  std::vector<unsigned long long> is, dr;
  for (int i = 0; i < grid * 8; ++i) {
    is.push_back(hs[2 * i]);
    dr.push_back(hs[2 * i + 1]);
  }
  std::sort(is.begin(), is.end());
  std::sort(dr.begin(), dr.end());
  const double us = ms * 1e3 / iters;
  const double bytes = (double)grid * kRows * 256 * 4 * kReps;  // output tile bytes
  std::printf("%-8s ld=%5d B grid=%4d: issue med %6llu p90 %6llu cyc, drain med %6llu p90 %6llu cyc per 128 KiB tile; "
              "kernel %7.1f us = %6.0f GB/s of tile, %5.1f B/cyc/CU at 2.2 GHz; %s\n",
              name, hLd * 4, grid, is[is.size() / 2], is[is.size() * 9 / 10], dr[dr.size() / 2], dr[dr.size() * 9 / 10], us,
              bytes / us / 1e3, bytes / grid / (us * 2200.0), bad ? "VALUES WRONG" : "values ok");
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return bad ? 1 : 0;
}

int main() {
  float* out;
  unsigned long long* st;
  CK(hipMalloc(&out, (size_t)kReps * 256 * kRows * 2048 * 4));
  CK(hipMalloc(&st, 256 * 16 * 8));
  int rc = 0;
  for (int ld : {1024, 1536}) {
    hLd = ld;
    for (int grid : {32, 256}) {
      rc |= run<STORE>("store", out, st, grid);
      rc |= run<STOREQ>("storeq", out, st, grid);
      rc |= run<RMW>("rmw", out, st, grid);
      rc |= run<RMWQ>("rmwq", out, st, grid);
      rc |= run<ATOM4>("atom4", out, st, grid);
      rc |= run<ATOMROW>("atomrow", out, st, grid);
    }
  }
  CK(hipFree(out));
  CK(hipFree(st));
  return rc;
}
