// Diagnostic only (never part of libcnmf_hip.so): the chip's streaming-read ceiling for the access
// shape of the persistent MU kernel.  Each workgroup reads whole contiguous tiles b, b + G, ... of
// 256·U 16-byte chunks, `passes` times over the buffer, with D register tile sets (probe_reg) or an
// S-slot LDS-DMA ring per wave (probe_lds, global_load_lds_dwordx4, no barriers: each wave reads
// back only its own pieces after its own counted vmcnt).  AUX: 0 = default policy, 2 = nt.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int AUX>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (AUX == 2) return __builtin_nontemporal_load(p);
  else return *p;
}

template <int U, int D, int AUX>
__global__ __launch_bounds__(256) void probe_reg(const u32x4* __restrict__ X, int nbt, int passes, unsigned* out) {
  const int G = gridDim.x, b = blockIdx.x, t = threadIdx.x;
  unsigned acc = 0;
  u32x4 r[D][U];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int u = 0; u < U; ++u) r[d][u] = ld16<AUX>(X + ((size_t)(b + (size_t)G * d) * U + u) * 256 + t);
  for (int p = 0; p < passes; ++p) {
    for (int i = 0; i < nbt; i += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= r[d][u].x ^ r[d][u].y ^ r[d][u].z ^ r[d][u].w;
        int nx = i + d + D;
        if (nx >= nbt) nx -= nbt;  // wraps into the next pass's first tiles
#pragma unroll
        for (int u = 0; u < U; ++u) r[d][u] = ld16<AUX>(X + ((size_t)(b + (size_t)G * nx) * U + u) * 256 + t);
      }
    }
  }
  if (acc == 0x12345678u) out[b] = acc;  // keeps the loads alive
}

template <int U, int S, int AUX>
__global__ __launch_bounds__(256) void probe_lds(const u32x4* __restrict__ X, int nbt, int passes, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int G = gridDim.x, b = blockIdx.x, t = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), l = t & 63;
  unsigned acc = 0;
  auto issue = [&](int tile_i, int slot) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32x4* src = X + ((size_t)(b + (size_t)G * tile_i) * U) * 256 + (w * U + u) * 64 + l;
      unsigned char* dst = smem + (((size_t)(w * S + slot) * U + u) * 64) * 16;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, AUX);
    }
  };
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s, s);
  int slot = 0;
  for (int p = 0; p < passes; ++p) {
    for (int i = 0; i < nbt; ++i) {
      int nx = i + S - 1;
      if (nx >= nbt) nx -= nbt;
      int ns = slot + S - 1;
      if (ns >= S) ns -= S;
      issue(nx, ns);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * (S - 1)) : "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(smem + ((((size_t)(w * S + slot) * U + u) * 64) + l) * 16);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
      slot = slot + 1 == S ? 0 : slot + 1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x12345678u) out[b] = acc;
}

using Fn = void (*)(const u32x4*, int, int, unsigned*);
struct K { const char* name; Fn fn; int U; int lds_per_wave; };
static const K kKernels[] = {
    {"reg_U4_D2", &probe_reg<4, 2, 0>, 4, 0},
    {"reg_U4_D2_nt", &probe_reg<4, 2, 2>, 4, 0},
    {"reg_U8_D2_nt", &probe_reg<8, 2, 2>, 8, 0},
    {"reg_U4_D4_nt", &probe_reg<4, 4, 2>, 4, 0},
    {"lds_U4_S3", &probe_lds<4, 3, 0>, 4, 3 * 4 * 1024},
    {"lds_U4_S3_nt", &probe_lds<4, 3, 2>, 4, 3 * 4 * 1024},
    {"lds_U4_S4_nt", &probe_lds<4, 4, 2>, 4, 4 * 4 * 1024},
    {"lds_U8_S3_nt", &probe_lds<8, 3, 2>, 8, 3 * 8 * 1024},
};

extern "C" {
int probe_count(void) { return (int)(sizeof(kKernels) / sizeof(kKernels[0])); }
const char* probe_name(int i) { return kKernels[i].name; }
int probe_U(int i) { return kKernels[i].U; }
int probe_launch(int i, const void* X, int grid, int nbt, int passes, unsigned* out, void* stream) {
  const K& k = kKernels[i];
  const size_t lds = (size_t)k.lds_per_wave * 4;
  if (lds > 0 && hipFuncSetAttribute((const void*)k.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -1;
  hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), lds, (hipStream_t)stream, (const u32x4*)X, nbt, passes, out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
}
