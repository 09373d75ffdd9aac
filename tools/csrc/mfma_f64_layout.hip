// Probe of the v_mfma_f64_4x4x4f64 (4 blocks) operand / result lane layout on gfx950: which lanes
// hold A[i][k], B[k][j] and D[i][j] of each 4x4 block.  Prints, per lane, D for A = lane id (B = 1)
// and for B = lane id (A = 1), and for the one-hot A / B sweeps the lanes that contribute.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double* out, int mode, int hot) {
  const int l = threadIdx.x;
  double a = 1.0, b = 1.0;
  if (mode == 0) a = (double)l;              // D = sum of the A lanes of its row
  if (mode == 1) b = (double)l;              // D = sum of the B lanes of its column
  if (mode == 2) { a = (l == hot) ? 1.0 : 0.0; b = 1.0; }
  if (mode == 3) { b = (l == hot) ? 1.0 : 0.0; a = 1.0; }
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  out[l] = d;
}

// issue cost: 4 independent chains of N instructions, cycles per instruction (one wave)
__global__ void timing(double* out, int which, int n) {
  const int l = threadIdx.x;
  double c0 = l, c1 = l + 1, c2 = l + 2, c3 = l + 3;
  const double a = 1.0000001 + l * 1e-9, b = 0.9999999;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (which == 0) {
    for (int i = 0; i < n; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
    }
  } else if (which == 1) {
    for (int i = 0; i < n; ++i) {
      c0 = fma(a, c0, b);
      c1 = fma(a, c1, b);
      c2 = fma(a, c2, b);
      c3 = fma(a, c3, b);
    }
  } else {
    typedef double d4 __attribute__((ext_vector_type(4)));
    d4 acc = {c0, c1, c2, c3};
    for (int i = 0; i < n; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    c0 = acc[0]; c1 = acc[1]; c2 = acc[2]; c3 = acc[3];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = c0 + c1 + c2 + c3;
  if (l == 0) out[64] = (double)(t1 - t0) / (4.0 * n);
}

int main() {
  double* d;
  hipMalloc(&d, 64 * sizeof(double));
  double h[64];
  for (int mode = 0; mode < 2; ++mode) {
    probe<<<1, 64>>>(d, mode, 0);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mode %d:", mode);
    for (int l = 0; l < 64; ++l) printf(" %g", h[l]);
    printf("\n");
  }
  // one-hot: for each source lane, the output lanes it reaches
  for (int mode = 2; mode < 4; ++mode) {
    printf("mode %d (%s one-hot -> D lanes):\n", mode, mode == 2 ? "A" : "B");
    for (int hot = 0; hot < 64; ++hot) {
      probe<<<1, 64>>>(d, mode, hot);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf(" src %2d:", hot);
      for (int l = 0; l < 64; ++l) if (h[l] != 0.0) printf(" %d", l);
      printf("\n");
    }
  }
  double* dt;
  hipMalloc(&dt, 65 * sizeof(double));
  const char* names[] = {"v_mfma_f64_4x4x4f64 (4 chains)", "v_fma_f64 (4 chains)", "v_mfma_f64_16x16x4f64 (1 chain, /4)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int which = 0; which < 3; ++which) {
      timing<<<1, 64>>>(dt, which, 4096);
      double hh[65];
      hipMemcpy(hh, dt, sizeof(hh), hipMemcpyDeviceToHost);
      printf("%s: %.2f cycles per instruction\n", names[which], which == 2 ? hh[64] * 4.0 : hh[64]);
    }
  hipFree(d);
  return 0;
}
