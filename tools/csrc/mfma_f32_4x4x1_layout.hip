// Probe of v_mfma_f32_4x4x1_16b_f32 (16 blocks, K = 1) on gfx950: for a one-hot A (or B) lane, the
// (lane, register) positions of D it reaches; and its issue cost (4 independent chains, one wave).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out, int mode, int hot) {
  const int l = threadIdx.x;
  float a = 1.f, b = 1.f;
  if (mode == 0) a = (l == hot) ? 1.f : 0.f;
  if (mode == 1) b = (l == hot) ? 1.f : 0.f;
  f4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[4 * l + r] = d[r];
}

__global__ void timing(float* out, int n) {
  const int l = threadIdx.x;
  f4 c0 = {1.f * l, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  const float a = 1.0000001f, b = 0.9999999f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = c0[0] + c1[1] + c2[2] + c3[3];
  if (l == 0) out[64] = (float)(t1 - t0) / (4.f * n);
}

int main() {
  float* d;
  hipMalloc(&d, 256 * sizeof(float));
  float h[256];
  for (int mode = 0; mode < 2; ++mode) {
    printf("%s one-hot -> D (lane.reg):\n", mode == 0 ? "A" : "B");
    for (int hot = 0; hot < 64; hot += (hot < 8 ? 1 : 4)) {
      probe<<<1, 64>>>(d, mode, hot);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf(" src %2d:", hot);
      for (int i = 0; i < 256; ++i) if (h[i] != 0.f) printf(" %d.%d", i / 4, i % 4);
      printf("\n");
    }
  }
  float* dt;
  hipMalloc(&dt, 65 * sizeof(float));
  for (int rep = 0; rep < 2; ++rep) {
    timing<<<1, 64>>>(dt, 4096);
    float hh[65];
    hipMemcpy(hh, dt, sizeof(hh), hipMemcpyDeviceToHost);
    printf("v_mfma_f32_4x4x1_16b_f32 (4 chains): %.2f cycles per instruction\n", hh[64]);
  }
  return 0;
}
