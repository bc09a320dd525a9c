// Standalone A/B harness for the bf16 attention kernel: compiles attention.hip
// directly so build-time variants (-DATTN_STAGES=, -DATTN_OCC=) can be timed
// side by side without touching the shipped library. Prints the average time of
// one C2-sized launch (B=32, 577 tokens, 16 heads x 64) and an output checksum
// (variants must agree to within bf16 rounding of the same math).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iaa-clip_amd/csrc -DATTN_STAGES=3 \
//         tools/attn_bench.hip -o /tmp/attn_s3 && /tmp/attn_s3 [B] [N] [variant]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../aa-clip_amd/csrc/attention.hip"

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32, N = argc > 2 ? atoi(argv[2]) : 577, H = 16, D = H * 64, reps = 50;
  const int variant = argc > 3 ? atoi(argv[3]) : 0;  // aaclip_set_attn_variant
  if (aaclip_set_attn_variant(variant)) return 3;
  const size_t nq = (size_t)B * N * 3 * D, no = (size_t)B * N * D;
  std::vector<uint16_t> h(nq);
  uint32_t x = 12345;
  for (size_t i = 0; i < nq; ++i) {  // ~N(0,1)-ish: sum of 4 uniforms, scaled
    float s = 0.f;
    for (int k = 0; k < 4; ++k) {
      x = x * 1664525u + 1013904223u;
      s += (x >> 8) * (1.0f / 16777216.0f) - 0.5f;
    }
    const float f = s * 1.7320508f;
    uint32_t u;
    std::memcpy(&u, &f, 4);
    h[i] = (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
  }
  uint16_t *dq, *dout;
  if (hipMalloc(&dq, nq * 2) != hipSuccess || hipMalloc(&dout, no * 2) != hipSuccess) return 1;
  if (hipMemcpy(dq, h.data(), nq * 2, hipMemcpyHostToDevice) != hipSuccess) return 1;
  for (int i = 0; i < 5; ++i)
    if (aaclip_attention(AACLIP_BF16, dq, dout, B, N, H, 64, 0, nullptr, 0, nullptr)) return 2;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(e0, nullptr);
    for (int i = 0; i < reps; ++i) aaclip_attention(AACLIP_BF16, dq, dout, B, N, H, 64, 0, nullptr, 0, nullptr);
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms / reps < best ? ms / reps : best;
  }
  std::vector<uint16_t> o(no);
  (void)hipMemcpy(o.data(), dout, no * 2, hipMemcpyDeviceToHost);
  double cs = 0.0;
  for (size_t i = 0; i < no; ++i) {
    uint32_t u = (uint32_t)o[i] << 16;
    float f;
    std::memcpy(&f, &u, 4);
    cs += (double)f * (double)((i % 97) + 1);
  }
  const double flop = 4.0 * B * (double)N * N * D;
  printf("variant=%d N=%d  %8.2f us  %7.1f TFLOP/s  checksum %.6e\n", variant, N, best * 1e3,
         flop / (best * 1e-3) / 1e12, cs);
  return 0;
}
