// cnmf_hip.hip — MI355X (gfx950, CDNA4) kernels + C ABI for the Frobenius multiplicative update.
//
// What runs per MU iteration (sklearn naming, X[N][F] samples-major):
//
//   mu_pass_kernel      ONE streaming pass over X and W (the ~all-bytes kernel):
//                       per 64-sample tile staged in LDS: num = X·Hᵀ, den = W·HHᵀ (+l1)(+l2·W),
//                       W <- W·(num/den) written back, then the accumulators [WᵀX | WᵀW] of the
//                       NEW W folded into per-workgroup fp64 partials.       (SK:526-631, SK:639-640)
//   reduce_kernel       deterministic fp64 column-sum of the per-workgroup partials (fixed slice
//                       order, ticket-elected last workgroup combines the slices) and, fused for a
//                       single GPU, the basis update in that last workgroup.
//   basis_update        H <- H·(WᵀX / ((WᵀW)·H (+l1)(+l2·H))) in fp64, then Ht / HHt for the next
//                       pass.                                                 (SK:634-728)
//
// SK:<line> = sklearn/decomposition/_nmf.py (1.7.2), the algorithm the reference declares
// (/root/reference/setup.py:26,30; the reference's own cnmf/__init__.py is empty).
//
// Design notes (MI355X-first; see DESIGN.md for the roofline numbers):
//  * the pass is HBM-bound (≈4 flop/B): each workgroup (4 waves) streams whole 64-sample tiles of X
//    (64·F contiguous elements) and W through 16-byte register loads issued one tile AHEAD of the
//    compute (the next tile is in flight while the current one is reduced), then stores them
//    verbatim to LDS; no HBM byte is read twice per iteration.
//  * per-sample work maps lane = sample (num, update); the outer-product accumulation maps
//    lane = feature (A phase), so the k×(F+k) accumulators live in registers for the whole
//    launch and only ONE fp64 partial row per workgroup reaches HBM.
//  * precision: per-tile fp32 accumulation (16 or 64 terms), fp64 running sums, fp64 cross-block
//    reduction and fp64 basis update (H is kept in fp64 on the device) so the fp32 path tracks the
//    fp64 CPU oracle (≤1e-5 rel. Frobenius after 500 iterations).
//  * grid = persistent, sized from the occupancy query so that ceil(tiles/blocks) rounds are
//    balanced; tiles are dealt round-robin so concurrently running workgroups stream neighbouring
//    addresses.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "cnmf_hip.h"

namespace cnmf {

constexpr int TS = 64;       // samples per tile
constexpr int NT = 256;      // threads per workgroup
constexpr int NWAVE = NT / 64;
constexpr int PF = 8;        // 16-byte chunks per thread held in registers for the next tile
constexpr int NSLICE = 64;   // max slices of the deterministic cross-block reduction
constexpr int RED_NT = 256;  // threads of the reduce / update workgroups
constexpr double EPS32 = 1.1920928955078125e-07;  // np.finfo(np.float32).eps, SK:39
constexpr int ALS_TAB = 16 * 16 + 16;  // constrained-ALS passive-set table: 16 masks x 4x4 + valid

static thread_local char g_err[512] = "";

static int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// Diagnostic switches (A/B timing and tools/ probes) are read from the environment only in the
// diagnostic build (-DCNMF_DIAG: python -m cnmf_amd.build --diag); the product library ignores the
// environment, so every plan's behaviour follows from its arguments alone.
static const char* diag_env(const char* name) {
#ifdef CNMF_DIAG
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

#define HIP_CHECK(expr)                                                                   \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return set_err(CNMF_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));        \
  } while (0)

// ------------------------------------------------------------------------------------------------
// element conversions: X storage type -> compute type
// ------------------------------------------------------------------------------------------------
struct bf16_t {
  uint16_t bits;
};

// native 16-byte vector (HIP's uint4 class type defeats SROA: the prefetch array went to scratch)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float to_c(float v) { return v; }
__device__ __forceinline__ double to_c(double v) { return v; }
__device__ __forceinline__ float to_c(bf16_t v) { return __uint_as_float(((uint32_t)v.bits) << 16); }

template <typename TX>
struct Compute;
template <>
struct Compute<float> {
  using T = float;
};
template <>
struct Compute<double> {
  using T = double;
};
template <>
struct Compute<bf16_t> {
  using T = float;
};

__host__ __device__ constexpr size_t align16(size_t b) { return (b + 15) & ~size_t(15); }

// LDS carve of the pass kernel (bytes); identical on host and device.  Every offset is 16-aligned.
struct PassLds {
  size_t region0;  // X tile [TS][F] (+4 zero elements), later the cross-wave reduction scratch
  size_t w;        // old-W tile, flat [ns][k]
  size_t wn;       // new-W tile, [TS][KP] (zero for j >= k and for invalid samples)
  size_t ht;       // Ht (compute type), [4*q][KP], rows >= F zero (q = ceil(F/4) per lane)
  size_t hht;      // HHt (fp64), [KP][KP]
  size_t zero;     // 16 zero bytes (source of the idle lanes of the A phase)
  size_t total;
};

__host__ __device__ inline int feat_per_wave(int F) { return (F + NWAVE - 1) / NWAVE; }

__host__ __device__ inline PassLds pass_lds(int F, int KP, size_t sx, size_t sc, size_t sh = 0) {
  if (sh == 0) sh = sc;  // Ht element size (fp64 for the constrained-ALS pass)
  PassLds L;
  size_t xb = align16(((size_t)TS * F + 4) * sx);
  size_t rb = (size_t)NWAVE * 64 * KP * sizeof(double);
  L.region0 = xb > rb ? xb : rb;
  L.w = L.region0;
  L.wn = L.w + align16((size_t)TS * KP * sc);
  L.ht = L.wn + align16((size_t)TS * KP * sc);
  L.hht = L.ht + align16((size_t)NWAVE * feat_per_wave(F) * KP * sh);
  L.zero = L.hht + align16((size_t)(KP == 4 ? ALS_TAB : KP * KP) * sizeof(double));
  L.total = L.zero + 16;
  return L;
}

// Geometry of one tile's contiguous byte ranges in X and W.
struct TileGeom {
  const unsigned char* xsrc;
  const unsigned char* wsrc;
  int ns;   // valid samples
  int nxf;  // full 16-byte chunks of X
  int nch;  // full chunks of X + W
  int rx;   // trailing X elements (partial chunk)
  int rw;   // trailing W elements
  int nwf;
};

template <typename TX, typename TC>
__device__ __forceinline__ TileGeom tile_geom(const TX* X, const TC* W, int64_t tile, int64_t n_rows,
                                              int F, int k) {
  TileGeom g;
  int64_t s0 = tile * TS;
  int64_t rem = n_rows - s0;
  g.ns = rem < TS ? (int)rem : TS;
  size_t xb = (size_t)g.ns * F * sizeof(TX);
  size_t wb = (size_t)g.ns * k * sizeof(TC);
  g.xsrc = reinterpret_cast<const unsigned char*>(X) + (size_t)s0 * F * sizeof(TX);
  g.wsrc = reinterpret_cast<const unsigned char*>(W) + (size_t)s0 * k * sizeof(TC);
  g.nxf = (int)(xb >> 4);
  g.nwf = (int)(wb >> 4);
  g.nch = g.nxf + g.nwf;
  g.rx = (int)((xb & 15) / sizeof(TX));
  g.rw = (int)((wb & 15) / sizeof(TC));
  return g;
}

// Issue this thread's 16-byte chunk loads of a tile.  Branch-free on purpose: chunks past the tile
// re-read chunk 0 (an L1/L2 hit) instead of sitting in a divergent `if` — guarded loads made hipcc
// put an `s_waitcnt vmcnt(0)` in front of every load, serialising the prefetch (and waiting on the
// previous tile's W stores).
template <int N, int I0 = 0, int I1 = N>
__device__ __forceinline__ void prefetch_tile(u32x4 (&pf)[N], const TileGeom& g, int t) {
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    const int c = t + NT * i;
    const size_t off = c < g.nxf ? 16 * (size_t)c : (c < g.nch ? 16 * (size_t)(c - g.nxf) : 0);
    const unsigned char* base = (c < g.nxf || c >= g.nch) ? g.xsrc : g.wsrc;
    pf[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + off));
  }
}

// Write one staged tile into LDS: the prefetched registers, any chunks beyond the register depth,
// and for a ragged last tile the element tails plus 4 zero elements after the last valid row (the
// padded feature reads of phase 1 multiply them by zero Ht rows, so they must not hold NaN bits).
template <typename TX, typename TC, int N>
__device__ __forceinline__ void stage_tile(unsigned char* smem, size_t w_off, const TileGeom& g,
                                           const u32x4 (&pf)[N], int t, int F) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int c = t + NT * i;
    if (c < g.nch) {
      unsigned char* dst = c < g.nxf ? smem + 16 * (size_t)c : smem + w_off + 16 * (size_t)(c - g.nxf);
      *reinterpret_cast<u32x4*>(dst) = pf[i];
    }
  }
  for (int c = t + NT * N; c < g.nch; c += NT) {
    const unsigned char* src = c < g.nxf ? g.xsrc + 16 * (size_t)c : g.wsrc + 16 * (size_t)(c - g.nxf);
    unsigned char* dst = c < g.nxf ? smem + 16 * (size_t)c : smem + w_off + 16 * (size_t)(c - g.nxf);
    *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(src);
  }
  if (g.ns < TS) {
    TX* sX = reinterpret_cast<TX*>(smem);
    TC* sW = reinterpret_cast<TC*>(smem + w_off);
    if (t < g.rx) {
      const int e = g.nxf * (16 / (int)sizeof(TX)) + t;
      sX[e] = reinterpret_cast<const TX*>(g.xsrc)[e];
    }
    if (t >= 64 && t - 64 < g.rw) {
      const int e = g.nwf * (16 / (int)sizeof(TC)) + (t - 64);
      sW[e] = reinterpret_cast<const TC*>(g.wsrc)[e];
    }
    if (t >= 128 && t - 128 < 4) sX[g.ns * F + (t - 128)] = TX{};
  }
}

template <typename T>
__device__ __forceinline__ T lds_at(const unsigned char* smem, uint32_t off) {
  return *reinterpret_cast<const T*>(smem + off);
}


// ------------------------------------------------------------------------------------------------
// Diagnostic phase stamps (built only with -DCNMF_STAMPS into a separate .so; never in the real
// kernel): per wave, s_memtime deltas between the phase boundaries of every tile are summed in
// registers and added once per wave into g_stamps[slot] (MI355X guide §7 "In-kernel stamps").
// ------------------------------------------------------------------------------------------------
#ifdef CNMF_STAMPS
__device__ unsigned long long g_stamps[16];
#define STAMP_DECL unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long st_t0 = 0;
#define STAMP(slot)                                                                   \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    unsigned long long st_t;                                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t) :: "memory");    \
    __builtin_amdgcn_sched_barrier(0);                                                \
    if (slot > 0) st_acc[slot] += st_t - st_t0;                                       \
    st_t0 = st_t;                                                                     \
  } while (0)
#define STAMP_FLUSH                                                                   \
  do {                                                                                \
    if ((threadIdx.x & 63) == 0)                                                      \
      for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_stamps[i_], st_acc[i_]);           \
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_stamps[8], 1ull);                       \
  } while (0)
// the end of a persistent bfw iteration: thread 0 of every workgroup sums the phase durations
// (s_memtime) into g_eoi[slot]; g_eoi[15] counts the (workgroup, iteration) pairs
__device__ unsigned long long g_eoi[16];
// the persistent ALS resume path of workgroup 0: per slot the sum over iterations of the
// s_memrealtime stamp (differences of the sums = summed phase durations); g_ph[15] counts
__device__ unsigned long long g_ph[16];
#define PH(slot)                                                                        \
  do {                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                                          \
      g_ph[slot] += __builtin_amdgcn_s_memrealtime();                                   \
      if (slot == 0) g_ph[15] += 1ull;                                                  \
    }                                                                                   \
  } while (0)
#define EOI_DECL unsigned long long eoi_t0 = 0;
#define EOI(slot)                                                                     \
  do {                                                                                \
    if (threadIdx.x == 0) {                                                           \
      unsigned long long st_t;                                                        \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t) :: "memory");  \
      if (slot > 0) atomicAdd(&g_eoi[slot], st_t - eoi_t0);                           \
      else atomicAdd(&g_eoi[15], 1ull);                                               \
      eoi_t0 = st_t;                                                                  \
    }                                                                                 \
  } while (0)
#else
#define STAMP_DECL
#define STAMP(slot) do {} while (0)
#define STAMP_FLUSH do {} while (0)
#define EOI_DECL
#define EOI(slot) do {} while (0)
#define PH(slot) do {} while (0)
#endif

// ------------------------------------------------------------------------------------------------
// Phases 1+2 of a tile, shared by both pass kernels; wave-local (wave w owns samples
// [16w, 16w+16), lane = (sample s = lane/4, feature quarter qtr = lane%4)) and in fp64.
//
// Precision: a long fp32 chain for the dot products num = x·Hᵀ leaves a rounding error that is
// nearly the SAME every iteration once H settles, so it drifts coherently instead of averaging out:
// 500 iterations of k=8 MU end 1.8e-5 (rel. Frobenius) from the fp64 oracle with 81-term fp32
// chains, 5.5e-7 with 7-term fp32 chains folded into fp64 (NumPy emulation of this kernel's
// arithmetic) — as good as all-fp64, at fp32 VALU cost.
//   phase 1: lane sums its quarter of x[s]·Ht (Ht rows >= F are zero) in fp32 chains of 7 folded
//            into fp64; quad shuffles in the fixed order (q0+q1)+(q2+q3) complete num[s][0..KP);
//   phase 2: lane (s, qtr) updates components j = qtr + 4c:
//            den = Σ_m w[s][m]·HHt[j][m] (+l1)(+l2·w), den==0 -> eps32, w' = w·(num/den) in fp64,
//            rounded once to TC, stored to HBM and to the LDS row sWn[s] (A phase input).
//   loss   : lane sums (x − w·Ht)² over its quarter, quad-reduced into loss64 (qtr 0 lanes).
// ------------------------------------------------------------------------------------------------
template <typename TX, typename TC, int KP, int FT, bool ALS = false,
          typename TH = typename std::conditional<ALS, double, TC>::type>
__device__ __forceinline__ void phase12(const TX* __restrict__ sX, const TC* __restrict__ sW,
                                        TC* __restrict__ sWn, const TH* __restrict__ sHt,
                                        const double* __restrict__ sHHt, TC* __restrict__ W,
                                        int64_t tile, int F, int q, int k, int ns, int s_beg,
                                        int lane, bool do_loss, bool do_upd, double l1, double l2,
                                        double& loss64) {
  const int qtr = lane & 3;
  const int s = s_beg + (lane >> 2);
  const int fb = qtr * q;
  const TX* xr = sX + (size_t)s * F + fb;
  const TH* hb = sHt + (size_t)fb * KP;
  if (do_loss) {
    double w[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) w[j] = (j < k && s < ns) ? (double)sW[s * k + j] : 0.0;
    const int nf = min(q, F - fb);
    double part = 0.0;
    for (int f = 0; f < nf; ++f) {
      double wh = 0.0;
#pragma unroll
      for (int j = 0; j < KP; ++j) wh = fma(w[j], (double)hb[f * KP + j], wh);
      const double r = (double)to_c(xr[f]) - wh;
      part = fma(r, r, part);
    }
    part += __shfl_xor(part, 1);
    part += __shfl_xor(part, 2);
    if (qtr == 0 && s < ns) loss64 += part;
    return;
  }
  // fp32 (TC) FMA chains of PCH features folded into fp64 (see the precision note above); the
  // constrained-ALS step forms c = Hx entirely in fp64 (its solve amplifies errors by cond(Q))
  constexpr int PCH = 7;
  double p[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) p[j] = 0.0;
  if constexpr (ALS) {
    for (int f = 0; f < q; ++f) {
      const double xv = (double)to_c(xr[f]);
#pragma unroll
      for (int j = 0; j < KP; ++j) p[j] = fma(xv, hb[f * KP + j], p[j]);
    }
  } else if constexpr (FT > 0) {
    constexpr int QF = (FT + NWAVE - 1) / NWAVE;
#pragma unroll 1
    for (int f0 = 0; f0 < QF; f0 += PCH) {
      TC pc[KP];
#pragma unroll
      for (int j = 0; j < KP; ++j) pc[j] = TC(0);
#pragma unroll
      for (int ff = 0; ff < PCH; ++ff) {
        if (f0 + ff < QF) {
          const TC xv = to_c(xr[f0 + ff]);
#pragma unroll
          for (int j = 0; j < KP; ++j) pc[j] = fma(xv, hb[(f0 + ff) * KP + j], pc[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < KP; ++j) p[j] += (double)pc[j];
    }
  } else {
    for (int f0 = 0; f0 < q; f0 += PCH) {
      TC pc[KP];
#pragma unroll
      for (int j = 0; j < KP; ++j) pc[j] = TC(0);
      const int fe = min(q, f0 + PCH);
      for (int f = f0; f < fe; ++f) {
        const TC xv = to_c(xr[f]);
#pragma unroll
        for (int j = 0; j < KP; ++j) pc[j] = fma(xv, hb[f * KP + j], pc[j]);
      }
#pragma unroll
      for (int j = 0; j < KP; ++j) p[j] += (double)pc[j];
    }
  }
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    p[j] += __shfl_xor(p[j], 1);
    p[j] += __shfl_xor(p[j], 2);
  }
  if (!do_upd) return;
  if constexpr (KP == 4 && ALS) {
    {
      // ---- constrained-ALS W-step (oracle/als_ref.py fcls_w): w = argmin_{w>=0}
      // ½wᵀQw - cᵀw with Q = HHᵀ + δ²11ᵀ, c = Hx + δ²1 (l1 carries δ²).  sHHt holds, per passive
      // set (mask 0..15), T = (Q_PP)⁻¹ scattered to 4x4 and a valid flag.  Lane qtr evaluates the
      // masks qtr, qtr+4, qtr+8, qtr+12; the least objective -½c·w among the non-negative
      // candidates wins (ties: lowest mask), chosen across the quad by shuffles.
      double c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = p[j] + l1;
      double bestf = 1.0;
      int bestm = 16;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int m = qtr + 4 * u;
        const double* T = sHHt + m * 16;
        double w[4];
        bool feas = sHHt[256 + m] != 0.0;
        double f = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double v = 0.0;
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) v = fma(T[r * 4 + cc], c[cc], v);
          w[r] = v;
          feas = feas && v >= 0.0;
          f = fma(c[r], v, f);
        }
        f *= -0.5;
        if (feas && (f < bestf || (f == bestf && m < bestm))) {
          bestf = f;
          bestm = m;
        }
      }
#pragma unroll
      for (int off = 1; off <= 2; off <<= 1) {
        const double of = __shfl_xor(bestf, off);
        const int om = __shfl_xor(bestm, off);
        if (of < bestf || (of == bestf && om < bestm)) {
          bestf = of;
          bestm = om;
        }
      }
      const double* T = sHHt + min(bestm, 15) * 16;
      double wn64 = 0.0;
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) wn64 = fma(T[qtr * 4 + cc], c[cc], wn64);
      TC wn = TC(0);
      if (s < ns && qtr < k) {
        wn = (TC)fmax(wn64, 0.0);
        W[(size_t)(tile * TS + s) * k + qtr] = wn;
      }
      sWn[s * KP + qtr] = wn;
      return;
    }
  }
  double wr[KP];
#pragma unroll
  for (int m = 0; m < KP; ++m)
    wr[m] = (k == KP) ? (double)sW[s * KP + m] : ((m < k) ? (double)sW[s * k + m] : 0.0);
#pragma unroll
  for (int c = 0; c < KP / 4; ++c) {
    const int j = qtr + 4 * c;
    const double num = qtr == 0 ? p[4 * c] : (qtr == 1 ? p[4 * c + 1] : (qtr == 2 ? p[4 * c + 2] : p[4 * c + 3]));
    const double wold = qtr == 0 ? wr[4 * c] : (qtr == 1 ? wr[4 * c + 1] : (qtr == 2 ? wr[4 * c + 2] : wr[4 * c + 3]));
    TC wn = TC(0);
    if (s < ns && j < k) {
      double den = 0.0;
#pragma unroll
      for (int m = 0; m < KP; ++m) den = fma(wr[m], sHHt[j * KP + m], den);  // HHt symmetric
      if (l1 > 0.0) den += l1;                    // SK:616-617
      if (l2 > 0.0) den = den + l2 * wold;        // SK:618-619
      if (den == 0.0) den = EPS32;                // SK:620
      wn = (TC)(wold * (num / den));              // SK:622-629
      W[(size_t)(tile * TS + s) * k + j] = wn;
    }
    sWn[s * KP + j] = wn;
  }
}

// ------------------------------------------------------------------------------------------------
// The fused sample pass.
//   TX: X storage (float / double / bf16_t), TC: compute + W type, KP: padded k (4/8/16),
//   FT: compile-time n_features (0 = runtime; the headline F=81 is specialised so every feature
//   loop unrolls with immediate LDS offsets), NPW: 64-lane feature passes held in registers per
//   wave, SPLIT: the A phase splits the tile's samples over the 4 waves (V <= 128) or splits the
//   passes over the waves (wide rows).
//
// Per 64-sample tile (4 barriers):
//   stage   prefetched registers -> LDS; issue the NEXT tile's 16-byte loads (in flight during the
//           rest of this tile)
//   phase 1 lane = sample, wave = quarter of the features: partial num[s][j] = Σ_f x[s][f]·Ht[f][j]
//   phase 2 element (s, j): num = Σ_waves partial; den = Σ_m w[s][m]·HHt[m][j] (+l1)(+l2·w);
//           den==0 -> eps32; w' = w·(num/den) -> HBM and LDS
//   phase 3 lane = virtual feature v: acc[j][v] += w'[s][j]·[x | w'][s][v] (fp32 registers for
//           the whole launch; combined across waves in fp64 at the end)
// ------------------------------------------------------------------------------------------------
// minimum waves per SIMD the register allocator must leave room for (no spills; measured with
// -Rpass-analysis=kernel-resource-usage): the F=81 fp32 k<=4 kernel fits 128 VGPRs (4 waves/SIMD)
template <typename TX, int KP, int FT>
constexpr int pass_min_waves() {
  return FT == 0 ? ((KP == 16 || sizeof(TX) == 8) ? 1 : 2)
                 : (KP == 4 ? (sizeof(TX) == 8 ? 3 : 4)
                            : (KP == 8 ? (sizeof(TX) == 8 ? 2 : 3) : (sizeof(TX) == 8 ? 1 : 2)));
}

template <typename TX, int KP, int FT, int NPW, bool SPLIT, bool ALS = false>
__global__ __launch_bounds__(NT, (pass_min_waves<TX, KP, FT>())) void mu_pass_kernel(const TX* __restrict__ X,
                                                     typename Compute<TX>::T* __restrict__ W,
                                                     const double* __restrict__ Ht,
                                                     const double* __restrict__ HHt,
                                                     double* __restrict__ partials, int64_t n_rows,
                                                     int F_rt, int k, double l1, double l2,
                                                     int flags, int64_t n_tiles) {
  using TC = typename Compute<TX>::T;
  using TH = typename std::conditional<ALS, double, TC>::type;  // Ht in LDS
  constexpr bool SAME = sizeof(TX) == sizeof(TC);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int F = FT > 0 ? FT : F_rt;
  const int q = feat_per_wave(F);
  const PassLds L = pass_lds(F, KP, sizeof(TX), sizeof(TC), sizeof(TH));
  TX* sX = reinterpret_cast<TX*>(smem);
  TC* sW = reinterpret_cast<TC*>(smem + L.w);
  TC* sWn = reinterpret_cast<TC*>(smem + L.wn);
  TH* sHt = reinterpret_cast<TH*>(smem + L.ht);
  double* sHHt = reinterpret_cast<double*>(smem + L.hht);
  double* sRed = reinterpret_cast<double*>(smem);

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int V = F + k;
  const int np = (V + 63) >> 6;
  const bool do_upd = (flags & CNMF_PASS_UPDATE_W) != 0;
  const bool do_acc = (flags & CNMF_PASS_ACCUMULATE) != 0;
  const bool do_loss = (flags & CNMF_PASS_LOSS) != 0;
  // basis-side constants into LDS once per launch (Ht zero-padded to 4q rows)
  for (int e = t; e < NWAVE * q * KP; e += NT) sHt[e] = e < F * KP ? (TH)Ht[e] : TH(0);
  const int n_hht = ALS ? ALS_TAB : KP * KP;  // HHt, or the ALS passive-set table
  for (int e = t; e < n_hht; e += NT) sHHt[e] = HHt[e];
  if (t < 4) {
    sX[TS * F + t] = TX{};
    reinterpret_cast<uint32_t*>(smem + L.zero)[t] = 0u;
  }

  TC acc[NPW][KP];
#pragma unroll
  for (int i = 0; i < NPW; ++i)
#pragma unroll
    for (int j = 0; j < KP; ++j) acc[i][j] = TC(0);
  double loss64 = 0.0;
  STAMP_DECL

  // 16-byte chunks per thread per tile: exact for a compile-time F, PF otherwise
  constexpr int PFT = FT > 0 ? (int)((TS * FT * sizeof(TX) + TS * KP * sizeof(TC) + 16 * NT - 1) / (16 * NT)) : PF;
  u32x4 pf[PFT];
  int64_t tile = blockIdx.x;
  if (tile < n_tiles) {
    TileGeom g = tile_geom(X, W, tile, n_rows, F, k);
    prefetch_tile<PFT>(pf, g, t);
  }

  for (; tile < n_tiles; tile += gridDim.x) {
    const TileGeom g = tile_geom(X, W, tile, n_rows, F, k);
    const int ns = g.ns;
    STAMP(0);
    stage_tile<TX, TC, PFT>(smem, L.w, g, pf, t, F);
    STAMP(1);  // 1: wait for this tile's loads + LDS writes
    __syncthreads();
    STAMP(2);  // 2: staging barrier

    // ---- issue the next tile's loads; they stay in flight through this tile's compute
    {
      const int64_t nt = tile + gridDim.x;
      if (nt < n_tiles) {
        prefetch_tile<PFT>(pf, tile_geom(X, W, nt, n_rows, F, k), t);
      }
    }
    STAMP(3);  // 3: prefetch issue

    // ---- phases 1+2 (wave-local, fp64)
    const int s_beg = wave * (TS / NWAVE);
    phase12<TX, TC, KP, FT, ALS>(sX, sW, sWn, sHt, sHHt, W, tile, F, q, k, ns, s_beg, lane, do_loss,
                                 do_upd, l1, l2, loss64);
    STAMP(4);  // 4: phases 1+2
    if (do_upd) {
      if (SPLIT)
        __builtin_amdgcn_wave_barrier();  // sWn rows of this wave feed its own A phase
      else
        __syncthreads();                  // wide rows: the A phase reads every wave's rows
    }

    if (do_acc) {
      // ---- phase 3: lane = virtual feature v (v < F: X column, F <= v < F+k: W_new column,
      //      beyond: a zero word); acc[j][v] += w_new[s][j]·value[s][v]  (SK:639-640)
      if (SPLIT) {
        const int nsw = min(max(ns - s_beg, 0), TS / NWAVE);
        // per-lane byte offset / stride of each pass's source column
        uint32_t offx[NPW], stx[NPW], offw[NPW], stw[NPW];
        bool isx[NPW];
#pragma unroll
        for (int i = 0; i < NPW; ++i) {
          const int v = 64 * i + lane;
          isx[i] = v < F;
          offx[i] = (uint32_t)((size_t)s_beg * F + min(v, F - 1)) * sizeof(TX);
          stx[i] = (uint32_t)(F * sizeof(TX));
          const bool isw = v >= F && v < V;
          offw[i] = isw ? (uint32_t)(L.wn + ((size_t)s_beg * KP + (v - F)) * sizeof(TC)) : (uint32_t)L.zero;
          stw[i] = isw ? (uint32_t)(KP * sizeof(TC)) : 0u;
        }
        auto body = [&](int s) {
          TC wv[KP];
#pragma unroll
          for (int j = 0; j < KP; ++j) wv[j] = sWn[(s_beg + s) * KP + j];
#pragma unroll
          for (int i = 0; i < NPW; ++i) {
            if (i < np) {
              TC val;
              if (64 * i + 64 <= F) {
                val = to_c(sX[(size_t)(s_beg + s) * F + 64 * i + lane]);
              } else if constexpr (SAME) {
                const uint32_t o = isx[i] ? offx[i] + s * stx[i] : offw[i] + s * stw[i];
                val = lds_at<TC>(smem, o);
              } else {
                const TC vx = to_c(lds_at<TX>(smem, offx[i] + s * stx[i]));
                const TC vw = lds_at<TC>(smem, offw[i] + s * stw[i]);
                val = isx[i] ? vx : vw;
              }
#pragma unroll
              for (int j = 0; j < KP; ++j) acc[i][j] = fma(wv[j], val, acc[i][j]);
            }
          }
        };
        if (nsw == TS / NWAVE) {
#pragma unroll 4
          for (int s = 0; s < TS / NWAVE; ++s) body(s);
        } else {
          for (int s = 0; s < nsw; ++s) body(s);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NPW; ++i) {
          const int p = wave + NWAVE * i;
          if (p < np) {
            const int v = 64 * p + lane;
            const bool full = 64 * p + 64 <= F;
            const bool isx = v < F;
            const uint32_t offx = (uint32_t)min(v, F - 1) * sizeof(TX);
            const bool isw = v >= F && v < V;
            const uint32_t offw = isw ? (uint32_t)(L.wn + (v - F) * sizeof(TC)) : (uint32_t)L.zero;
            const uint32_t stw = isw ? (uint32_t)(KP * sizeof(TC)) : 0u;
#pragma unroll 4
            for (int s = 0; s < ns; ++s) {
              TC wv[KP];
#pragma unroll
              for (int j = 0; j < KP; ++j) wv[j] = sWn[s * KP + j];
              TC val;
              if (full) {
                val = to_c(sX[(size_t)s * F + v]);
              } else {
                const TC vx = to_c(lds_at<TX>(smem, offx + (uint32_t)(s * F * sizeof(TX))));
                const TC vw = lds_at<TC>(smem, offw + s * stw);
                val = isx ? vx : vw;
              }
#pragma unroll
              for (int j = 0; j < KP; ++j) acc[i][j] = fma(wv[j], val, acc[i][j]);
            }
          }
        }
      }
    }
    STAMP(5);  // 5: phase 3
    __syncthreads();  // LDS tiles are rewritten by the next iteration
    STAMP(6);  // 6: end-of-tile barrier
  }
  STAMP_FLUSH;

  // ---- per-workgroup partial rows (fp64 combine of the 4 waves' fp32 accumulators)
  if (do_acc) {
    const int n_out = k * V;
    double* prow = partials + (size_t)blockIdx.x * n_out;
    if (SPLIT) {
#pragma unroll
      for (int i = 0; i < NPW; ++i) {
        if (i < np) {
          __syncthreads();
#pragma unroll
          for (int j = 0; j < KP; ++j) sRed[(wave * 64 + lane) * KP + j] = (double)acc[i][j];
          __syncthreads();
          for (int e = t; e < 64 * KP; e += NT) {
            const int l = e & 63;
            const int j = e >> 6;
            const int v = 64 * i + l;
            if (v < V && j < k) {
              const double sum = ((sRed[(0 * 64 + l) * KP + j] + sRed[(1 * 64 + l) * KP + j]) +
                                  sRed[(2 * 64 + l) * KP + j]) + sRed[(3 * 64 + l) * KP + j];
              prow[j * V + v] = sum;
            }
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NPW; ++i) {
        const int p = wave + NWAVE * i;
        const int v = 64 * p + lane;
        if (p < np && v < V) {
#pragma unroll
          for (int j = 0; j < KP; ++j)
            if (j < k) prow[j * V + v] = (double)acc[i][j];
        }
      }
    }
  }
  if (do_loss) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) loss64 += __shfl_xor(loss64, off);
    __syncthreads();
    if (lane == 0) sRed[wave] = loss64;
    __syncthreads();
    if (t == 0) partials[blockIdx.x] = ((sRed[0] + sRed[1]) + sRed[2]) + sRed[3];
  }
}

// ------------------------------------------------------------------------------------------------
// The fused sample pass on the matrix cores (fp32 compute; X fp32 or bf16; V = F + k <= 128).
//
// Same tile pipeline as mu_pass_kernel (64-sample tiles, register prefetch one tile ahead, 2
// barriers per tile); each wave owns 16 samples and runs its two small GEMMs on
// v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf chain, MI355X_MICROARCH.md §Matrix cores):
//   phase 1  num[j][s]  = Σ_f Ht[f][j]·x[s][f]      M = j (16, KP used), N = 16 samples,
//                                                    K = F in steps of 4; the Ht operand lives in
//                                                    VGPRs for the whole launch
//   phase 2  lane (s, j-group) applies the MU update to 4 components (W <- W·num/den)
//   phase 3  acc[j][v] += Σ_s w'[s][j]·[x | w'][s][v] M = j, N = V in 16-column blocks,
//                                                    K = the wave's 16 samples
// The accumulators stay in registers for the whole launch; the 4 waves are combined in fp64 at
// the end exactly like mu_pass_kernel (same partial-row layout [k][F+k]).
// ------------------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NB_MAX = 8;  // 16-column blocks of [X | W'] (V <= 128)

template <typename TX, int KP, int FT>
__global__ __launch_bounds__(NT, FT > 0 ? (KP == 16 ? 2 : (KP == 8 ? 3 : 4)) : 2) void mu_pass_mfma_kernel(const TX* __restrict__ X,
                                                            float* __restrict__ W,
                                                            const double* __restrict__ Ht,
                                                            const double* __restrict__ HHt,
                                                            double* __restrict__ partials,
                                                            int64_t n_rows, int F_rt, int k, double l1,
                                                            double l2, int flags, int64_t n_tiles) {
  using TC = float;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int F = FT > 0 ? FT : F_rt;
  const int V = F + k;
  const int nb_cnt = (V + 15) >> 4;    // phase-3 column blocks
  const PassLds L = pass_lds(F, KP, sizeof(TX), sizeof(TC));
  TX* sX = reinterpret_cast<TX*>(smem);
  TC* sW = reinterpret_cast<TC*>(smem + L.w);
  TC* sWn = reinterpret_cast<TC*>(smem + L.wn);
  TC* sHt = reinterpret_cast<TC*>(smem + L.ht);
  double* sHHt = reinterpret_cast<double*>(smem + L.hht);
  double* sRed = reinterpret_cast<double*>(smem);

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int ln = lane & 15;  // MFMA row/column index of this lane
  const int lk = lane >> 4;  // MFMA k index of this lane (and C/D row group)
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int s_beg = wave * (TS / NWAVE);
  const bool do_upd = (flags & CNMF_PASS_UPDATE_W) != 0;
  const bool do_acc = (flags & CNMF_PASS_ACCUMULATE) != 0;

  for (int e = t; e < NWAVE * feat_per_wave(F) * KP; e += NT) sHt[e] = e < F * KP ? (TC)Ht[e] : TC(0);
  for (int e = t; e < KP * KP; e += NT) sHHt[e] = HHt[e];
  if (t < 4) {
    sX[TS * F + t] = TX{};
    reinterpret_cast<uint32_t*>(smem + L.zero)[t] = 0u;
  }
  // column blocks held in registers: exact for a compile-time F (k <= KP), NB_MAX otherwise
  constexpr int NBC = FT > 0 ? (FT + KP + 15) / 16 : NB_MAX;
  f32x4 acc[NBC];
#pragma unroll
  for (int nb = 0; nb < NBC; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int PFT = FT > 0 ? (int)((TS * FT * sizeof(TX) + TS * KP * sizeof(TC) + 16 * NT - 1) / (16 * NT)) : PF;
  u32x4 pf[PFT];
  int64_t tile = blockIdx.x;
  if (tile < n_tiles) prefetch_tile<PFT>(pf, tile_geom(X, W, tile, n_rows, F, k), t);

  for (; tile < n_tiles; tile += gridDim.x) {
    const TileGeom g = tile_geom(X, W, tile, n_rows, F, k);
    const int ns = g.ns;
    stage_tile<TX, TC, PFT>(smem, L.w, g, pf, t, F);
    __syncthreads();
    {
      const int64_t nt = tile + gridDim.x;
      if (nt < n_tiles) prefetch_tile<PFT>(pf, tile_geom(X, W, nt, n_rows, F, k), t);
    }

    // ---- phases 1+2 (wave-local, fp64; shared with mu_pass_kernel)
    double loss_unused = 0.0;
    phase12<TX, TC, KP, FT>(sX, sW, sWn, sHt, sHHt, W, tile, F, feat_per_wave(F), k, ns, s_beg, lane,
                            false, do_upd, l1, l2, loss_unused);
    if (do_upd) __builtin_amdgcn_wave_barrier();  // this wave's sWn rows feed its own phase 3

    if (do_acc) {
      // ---- phase 3: acc[nb][r] = Σ_s w'[s][4lk+r]·val[s][16nb+ln]
#pragma unroll 2
      for (int st = 0; st < TS / NWAVE / 4; ++st) {
        const int ss = s_beg + 4 * st + lk;
        const bool sv = ss < ns;
        const float a3 = ln < KP ? sWn[ss * KP + min(ln, KP - 1)] : 0.0f;
#pragma unroll
        for (int nb = 0; nb < NBC; ++nb) {
          if (nb < nb_cnt) {
            const int v = 16 * nb + ln;
            float b3;
            if (16 * nb + 16 <= F) {
              b3 = to_c(sX[(size_t)ss * F + v]);
            } else {
              const float vx = to_c(sX[(size_t)ss * F + min(v, F - 1)]);
              const float vw = sWn[ss * KP + min(max(v - F, 0), KP - 1)];
              b3 = v < F ? vx : (v < V ? vw : 0.0f);
            }
            b3 = sv ? b3 : 0.0f;
            acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a3, b3, acc[nb], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();  // LDS tiles are rewritten by the next iteration
  }

  // ---- per-workgroup partial rows: D3[j = 4lk + r][v = 16nb + ln], 4 waves summed in fp64
  if (do_acc) {
    const int n_out = k * V;
    double* prow = partials + (size_t)blockIdx.x * n_out;
#pragma unroll
    for (int nb = 0; nb < NBC; ++nb) {
      if (nb < nb_cnt) {
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) sRed[(wave * 64 + lane) * 4 + r] = (double)acc[nb][r];
        __syncthreads();
        const int l = t & 63;
        const int r = t >> 6;
        const int j = 4 * (l >> 4) + r;
        const int v = 16 * nb + (l & 15);
        if (j < k && v < V) {
          const double sum = ((sRed[(0 * 64 + l) * 4 + r] + sRed[(1 * 64 + l) * 4 + r]) +
                              sRed[(2 * 64 + l) * 4 + r]) + sRed[(3 * 64 + l) * 4 + r];
          prow[j * V + v] = sum;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// The bf16 matrix-core pass (X bf16, F = 300, k = 16; any F % 4 == 0,
// F <= 384, 9 <= k <= 16).  One workgroup = 4 waves, 64-sample tiles, register prefetch one tile
// ahead (as mu_pass_kernel).  Both per-sample products run on v_mfma_f32_16x16x32_bf16:
//   phase 1  num[s][n] = Σ_f x[s][f]·H[n][f]   wave = 16 samples (M), N = 16 components, K = F in
//            steps of 32; A = X rows (ds_read_b64 pairs), B = H rows from LDS (ds_read_b128).
//   phase 2  lane = (4 samples, component): den = Σ_m w[s][m]·HHt[n][m] (fp64), the MU update
//            (SK:526-631) in fp64, W' -> HBM and to LDS transposed (W'ᵀ [16][68] fp32).
//   phase 3  acc[m][f] += Σ_s w'[s][m]·x[s][f]   M = 16 components, K = the tile's 64 samples, N =
//            the wave's 16-feature blocks (nb ≡ wave mod 4); B = X columns via ds_read_b64_tr_b16
//            (the hardware transpose read, one image for row and column reads); and
//            B[m][n] += Σ_s w'[s][m]·w'[s][n] on v_mfma_f32_16x16x4_f32 (the wave's 16 samples).
// Precision: X is exact in bf16; H and W' are each split into three bf16 terms (h = h1+h2+h3 to
// ~2^-27 relative) so every product X·h_i is exact in fp32, and each tile's fp32 MFMA sums are
// folded into fp64 accumulators (the 1e-5 bar of DESIGN.md §Precision).
// ------------------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef double f64x4 __attribute__((ext_vector_type(4)));

namespace bm {
constexpr int KP = 16;
constexpr int PFN = 11;      // 16-byte chunks per thread prefetched (tiles up to 44 KB: F <= 320)
constexpr int NBW_MAX = 5;   // 16-feature blocks per wave in phase 3 (F <= 320)
constexpr int WNT_ROW = 68;  // W'ᵀ row stride in floats (conflict-free transposed writes)
struct Lds {
  int x, w, wnt, hs, hht, total, hrow;  // byte offsets; hrow = bytes per H-split row
};
__host__ __device__ inline int ksteps(int F) { return (F + 31) / 32; }
__host__ __device__ inline Lds lds(int F) {
  Lds L;
  L.x = 0;
  L.w = (int)align16((size_t)TS * F * 2 + 64);        // + 64 zero bytes for the padded reads
  L.wnt = L.w + TS * KP * 4;
  L.hs = L.wnt + KP * WNT_ROW * 4;
  L.hrow = (32 * ksteps(F) + 8) * 2;                   // +16 B: conflict-free b128 row reads
  L.hht = L.hs + 3 * KP * L.hrow;
  L.total = L.hht + KP * KP * 8;
  return L;
}
__device__ __forceinline__ uint16_t bf16_rn(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf16_f(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }
}  // namespace bm

__global__ __launch_bounds__(NT, 2) void mu_pass_bf16_mfma_kernel(const bf16_t* __restrict__ X,
                                                                 float* __restrict__ W,
                                                                 const double* __restrict__ Ht,
                                                                 const double* __restrict__ HHt,
                                                                 double* __restrict__ partials,
                                                                 int64_t n_rows, int F, int k, double l1,
                                                                 double l2, int flags, int64_t n_tiles) {
  using namespace bm;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Lds L = lds(F);
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = lane >> 4;   // 16-lane group
  const int li = lane & 15;  // index inside the group
  const int KS = ksteps(F);
  const int NB = (F + 15) / 16;
  const bool do_upd = (flags & CNMF_PASS_UPDATE_W) != 0;
  const bool do_acc = (flags & CNMF_PASS_ACCUMULATE) != 0;
  float* sWnT = reinterpret_cast<float*>(smem + L.wnt);
  double* sHHt = reinterpret_cast<double*>(smem + L.hht);

  // ---- basis constants: H split into three bf16 rows [n][32·KS] (zero beyond F / k), HHt
  for (int e = t; e < KP * 32 * KS; e += NT) {
    const int n = e / (32 * KS);
    const int f = e - n * 32 * KS;
    const double h = (n < k && f < F) ? Ht[(size_t)f * KP + n] : 0.0;
    const uint16_t h1 = bf16_rn((float)h);
    const double r1 = h - (double)bf16_f(h1);
    const uint16_t h2 = bf16_rn((float)r1);
    const double r2 = r1 - (double)bf16_f(h2);
    const uint16_t h3 = bf16_rn((float)r2);
    uint16_t* row = reinterpret_cast<uint16_t*>(smem + L.hs + n * L.hrow) + f;  // split i at +i·KP rows
    row[0] = h1;
    row[KP * L.hrow / 2] = h2;
    row[2 * KP * L.hrow / 2] = h3;
  }
  for (int e = t; e < KP * KP; e += NT) sHHt[e] = HHt[e];
  for (int e = t; e < 16; e += NT) reinterpret_cast<uint32_t*>(smem + L.x + TS * F * 2)[e] = 0u;
  __syncthreads();
  double hhb[4];  // B operand of the den MFMA: HHᵀ[m = 4kk + g][n = li] (HHᵀ symmetric)
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) hhb[kk] = sHHt[(4 * kk + g) * KP + li];

  // phase 3 accumulators (A part: the wave's feature blocks; B part) in fp64, per-tile fp32 MFMA sums
  double acc64[NBW_MAX][4];
  double bacc64[4];
#pragma unroll
  for (int i = 0; i < NBW_MAX; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc64[i][r] = 0.0;
#pragma unroll
  for (int r = 0; r < 4; ++r) bacc64[r] = 0.0;

  u32x4 pf[PFN];
  STAMP_DECL
  int64_t tile = blockIdx.x;
  if (tile < n_tiles) prefetch_tile<PFN>(pf, tile_geom(X, W, tile, n_rows, F, k), t);

  for (; tile < n_tiles; tile += gridDim.x) {
    STAMP(0);
    const TileGeom gm = tile_geom(X, W, tile, n_rows, F, k);
    const int ns = gm.ns;
    stage_tile<bf16_t, float, PFN>(smem, L.w, gm, pf, t, F);
    STAMP(1);  // 1: wait for this tile's loads + LDS writes
    if (ns < TS) {  // ragged tile: rows >= ns must hold finite values for the MFMA reads
      uint16_t* sx = reinterpret_cast<uint16_t*>(smem + L.x);
      for (int e = ns * F + 4 + t; e < TS * F; e += NT) sx[e] = 0;
    }
    __syncthreads();
    STAMP(2);  // 2: staging barrier
    // the next tile's loads in two halves (here and after phase 1): issuing all eleven 16-byte
    // loads per thread at once stalled the issue on vector-memory back-pressure
    // (profiles/r02/session5/diag2/stamps_bf16.log)
    const int64_t nxt = tile + gridDim.x;
    const TileGeom gnx = tile_geom(X, W, nxt < n_tiles ? nxt : tile, n_rows, F, k);
    if (nxt < n_tiles) prefetch_tile<PFN, 0, PFN / 2>(pf, gnx, t);
    STAMP(3);  // 3: prefetch issue

    // ---- phase 1: num for samples 16·wave + (4g + r), component li
    f32x4 num;
    double num64[4] = {0.0, 0.0, 0.0, 0.0};
    {
      const unsigned char* xa = smem + L.x + ((size_t)(16 * wave + li) * F + 8 * g) * 2;
      const unsigned char* hb = smem + L.hs + li * L.hrow + 16 * g;
      for (int ks = 0; ks < KS; ++ks) {
        const uint64_t a0 = *reinterpret_cast<const uint64_t*>(xa + 64 * ks);
        const uint64_t a1 = *reinterpret_cast<const uint64_t*>(xa + 64 * ks + 8);
        s16x8 a;
        a.s0123 = __builtin_bit_cast(s16x4, a0);
        a.s4567 = __builtin_bit_cast(s16x4, a1);
        const s16x8 b1 = *reinterpret_cast<const s16x8*>(hb + 64 * ks);
        const s16x8 b2 = *reinterpret_cast<const s16x8*>(hb + KP * L.hrow + 64 * ks);
        const s16x8 b3 = *reinterpret_cast<const s16x8*>(hb + 2 * KP * L.hrow + 64 * ks);
        const bf16x8 av = __builtin_bit_cast(bf16x8, a);
        num = f32x4{0.f, 0.f, 0.f, 0.f};
        num = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, b3), num, 0, 0, 0);
        num = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, b2), num, 0, 0, 0);
        num = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, b1), num, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) num64[r] += (double)num[r];
      }
    }

    if (nxt < n_tiles) prefetch_tile<PFN, PFN / 2, PFN>(pf, gnx, t);
    STAMP(4);  // 4: phase 1
    // ---- phase 2: MU update of w[s][n], s = 16·wave + 4g + r, n = li (SK:526-631).
    // den = W·HHᵀ on v_mfma_f64_16x16x4_f64 (exact fp64 products and sums; f64 C/D layout: row =
    // g + 4·reg): its A-operand row ρ carries sample 4(ρ&3) + (ρ>>2), so D[g + 4r] is sample 4g + r,
    // the lane mapping of num.  HHᵀ (the B operand) lives in 4 registers per lane (hhb).
    if (do_upd) {
      const float* sWo = reinterpret_cast<const float*>(smem + L.w);
      f64x4 den = f64x4{0.0, 0.0, 0.0, 0.0};
      const int sa = 16 * wave + 4 * (li & 3) + (li >> 2);  // A-operand row li's sample
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int m = 4 * kk + g;
        const double a = m < k ? (double)sWo[sa * k + m] : 0.0;
        den = __builtin_amdgcn_mfma_f64_16x16x4f64(a, hhb[kk], den, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int s = 16 * wave + 4 * g + r;
        float wn = 0.f;
        if (s < ns && li < k) {
          double d = den[r];
          const double wold = (double)sWo[s * k + li];
          if (l1 > 0.0) d += l1;              // SK:616-617
          if (l2 > 0.0) d = d + l2 * wold;    // SK:618-619
          if (d == 0.0) d = EPS32;            // SK:620
          wn = (float)(wold * (num64[r] / d));  // SK:622-629
          W[(size_t)(tile * TS + s) * k + li] = wn;
        }
        sWnT[li * WNT_ROW + s] = wn;
      }
    }
    __syncthreads();  // every wave's W'ᵀ rows feed every wave's phase 3
    STAMP(5);  // 5: phase 2 + barrier

    // ---- phase 3: acc[m = 4g + r][f = 16·nb + li] += Σ_s w'[s][m]·x[s][f]; B on f32 MFMA
    if (do_acc) {
      f32x4 cacc[NBW_MAX];
#pragma unroll
      for (int i = 0; i < NBW_MAX; ++i) cacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int ks2 = 0; ks2 < 2; ++ks2) {
        // A operand: W'ᵀ[m = li][s = 32·ks2 + 8g + j], split into three bf16 terms
        const float* wr = sWnT + li * WNT_ROW + 32 * ks2 + 8 * g;
        const float4 w0 = *reinterpret_cast<const float4*>(wr);
        const float4 w1 = *reinterpret_cast<const float4*>(wr + 4);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        s16x8 a1, a2, a3;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint16_t h1 = bf16_rn(wv[j]);
          const float r1 = wv[j] - bf16_f(h1);
          const uint16_t h2 = bf16_rn(r1);
          const float r2 = r1 - bf16_f(h2);
          a1[j] = (short)h1;
          a2[j] = (short)h2;
          a3[j] = (short)bf16_rn(r2);
        }
        // B operand: X[s = 32·ks2 + 8g + j][f = 16·nb + li] by two transposed reads (4 rows each)
        const int q = li >> 2, p = li & 3;
        const unsigned char* xb0 = smem + L.x + ((size_t)(32 * ks2 + 8 * g + q) * F + 4 * p) * 2;
#pragma unroll
        for (int i = 0; i < NBW_MAX; ++i) {
          const int nb = wave + 4 * i;
          if (nb < NB) {
            const unsigned char* xb = xb0 + 32 * nb;
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xb));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xb + (size_t)4 * F * 2));
            s16x8 b;
            b.s0123 = lo;
            b.s4567 = hi;
            const bf16x8 bv = __builtin_bit_cast(bf16x8, b);
            cacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a3), bv, cacc[i], 0, 0, 0);
            cacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a2), bv, cacc[i], 0, 0, 0);
            cacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a1), bv, cacc[i], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < NBW_MAX; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc64[i][r] += (double)cacc[i][r];
      // B part: the wave's 16 samples, K = 4 per f32 MFMA (A = B operand value: W'ᵀ[li][s])
      f32x4 bacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const float v = sWnT[li * WNT_ROW + 16 * wave + 4 * kk + g];
        bacc = __builtin_amdgcn_mfma_f32_16x16x4f32(v, v, bacc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) bacc64[r] += (double)bacc[r];
    }
    __syncthreads();  // LDS tiles are rewritten by the next iteration
    STAMP(6);  // 6: phase 3 + end barrier
  }
  STAMP_FLUSH;

  // ---- per-workgroup partial row [k][F + k]: A from each wave's own blocks, B summed over waves
  if (do_acc) {
    const int V = F + k;
    double* prow = partials + (size_t)blockIdx.x * k * V;
#pragma unroll
    for (int i = 0; i < NBW_MAX; ++i) {
      const int nb = wave + 4 * i;
      const int f = 16 * nb + li;
      if (nb < NB && f < F) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 4 * g + r;
          if (m < k) prow[(size_t)m * V + f] = acc64[i][r];
        }
      }
    }
    double* red = reinterpret_cast<double*>(smem + L.x);
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wave * 64 + lane) * 4 + r] = bacc64[r];
    __syncthreads();
    {
      const int l = t & 63, r = t >> 6;  // output B[m = 4(l>>4) + r][n = l & 15]
      const int m = 4 * (l >> 4) + r, n = l & 15;
      if (m < k && n < k) {
        const double sum = ((red[(0 * 64 + l) * 4 + r] + red[(1 * 64 + l) * 4 + r]) +
                            red[(2 * 64 + l) * 4 + r]) + red[(3 * 64 + l) * 4 + r];
        prow[(size_t)m * V + F + n] = sum;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// mu_pass_bfw_kernel — the bf16 matrix-core pass of cfg4 (bf16 X, 9 <= k <= 16, F <= 320) as
// barrier-free WAVE tiles (mu_iter_wt_kernel's layout).
//
// mu_pass_bf16_mfma_kernel above shares each 64-sample tile among the workgroup's four waves and
// synchronises them three times per tile (staging, W'ᵀ hand-off, end of tile): at 2 waves per SIMD
// it ran latency-bound at 0.49 of HBM with 17 % MFMA busy and 16 % of cycles in LDS bank conflicts
// (profiles/r02/pmc_cfg/SUMMARY.md).  Here every wave owns a quarter of each of its workgroup's
// 64-sample tiles (16 samples, 9600 B of X at F = 300) and runs the whole update on it alone:
//   * prefetch: PD = 2 wave tiles in flight, X (10 x 16 B per lane) and W (one 16-byte chunk) loaded
//     by inline asm into AGPRs and waited for with exact counted `s_waitcnt vmcnt` (every body issues
//     exactly four stores, invalid lanes to a dummy word in this workgroup's partial row), staged into
//     the wave's own LDS slot: no barrier anywhere in the loop;
//   * phase 1  num[s][n] = Σ_f x[s][f]·h[n][f] on v_mfma_f32_16x16x32_bf16 (A = X rows, B = the three
//     bf16 terms of H, one fp32 chain per K-step folded into fp64) — as the 64-sample kernel;
//   * phase 2  den = w·HHᵀ on v_mfma_f64_16x16x4_f64, the fp64 update (SK:553-629); the lane's four
//     new w'[4g + r][li] are exactly the A operand of phase 3 (row m = li, k = samples 4g..4g+3), so
//     W' never goes through LDS;
//   * phase 3  A[m][f] += Σ_s w'[s][m]·x[s][f] on v_mfma_f32_16x16x16_bf16 (K = the tile's 16 samples;
//     B = X columns by ds_read_b64_tr_b16; w' in two bf16 terms since round 5 — 16 significant bits,
//     the dropped term an unbiased per-sample rounding that the sum over samples averages out);
//     B[m][n] += Σ_s w'[s][m]·w'[s][n] on v_mfma_f32_16x16x4_f32.  The fp32 MFMA accumulators chain
//     over the wave's tiles (≈ 61 at cfg4: the per-lane fp32 accumulation of mu_iter_wt_kernel);
//   * end of launch: the four waves' accumulators summed in LDS in the fixed order (w0 + w2) + (w1 + w3)
//     in fp64, one partial row per workgroup (mu_pass_bf16_mfma_kernel's row layout).
// Full 64-sample tiles only (the host runs a ragged tail on one workgroup of the 64-sample kernel).
// ------------------------------------------------------------------------------------------------
namespace bw {
constexpr int TSW = 16;       // samples per wave tile
constexpr int PFX = 10;       // 16-byte X loads per lane per wave tile (2F chunks, F <= 320)
constexpr int PFS = PFX + 1;  // + the wave tile's W (64k bytes: one chunk per lane, k <= 16)
constexpr int PD = 2;         // wave tiles in flight per wave
constexpr int NBX = 20;       // 16-feature blocks (F <= 320)
constexpr int NSTB = 4;       // global stores per body (the lane's four w')
struct Lds {
  int hs, hrow, hht, slot, xrow, xbytes, slotb, red, total;
};
// X row stride in a slot: the least multiple of 32 bytes >= 2F with an odd quotient (≡ 32, 96, 160 or
// 224 mod 256: 608 at F = 300).  Row ρ then starts on dword 8·odd·ρ mod 64, so phase 1's ds_read_b128
// row reads (rows li, 16-B columns g: groups of 16 lanes) and phase 3's transposed reads (rows 4g + q,
// 8-B columns pp) fall on distinct banks; the packed 600-B rows were 2- and 3-way conflicted.
__host__ __device__ inline int xrow_stride(int F) {
  int r = (2 * F + 31) / 32;
  if ((r & 1) == 0) ++r;
  return 32 * r;
}
__host__ __device__ inline Lds lds(int F) {
  Lds L;
  L.hrow = xrow_stride(32 * bm::ksteps(F));            // H split rows: the same rule, for the b128 reads
  L.hs = 0;
  L.hht = L.hs + 3 * bm::KP * L.hrow;
  L.xrow = xrow_stride(F);
  L.xbytes = (int)align16((size_t)TSW * L.xrow + 64);  // + 64 zero bytes for the reads past the last row
  L.slotb = L.xbytes + TSW * 16 * 4;                   // + the wave tile's W [16][k <= 16] fp32
  L.slot = (int)align16((size_t)L.hht + 16 * 16 * 8);
  L.red = 4 * ((NBX + 2) / 2) * 4 * 64 * 8;            // end of an iteration: four waves' fp64 sums, half the blocks
  const int loop = L.slot + 8 * L.slotb;  // two wave-tile slots per wave
  L.total = loop > L.red ? loop : L.red;
  return L;
}
__device__ __forceinline__ void ld16(u32x4& r, const unsigned char* p) {
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=a"(r) : "v"(p) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_set(u32x4 (&pf)[PFS]) {
  static_assert(PFS == 11, "one operand per prefetch register");
  asm volatile("s_waitcnt vmcnt(%11)"
               : "+a"(pf[0]), "+a"(pf[1]), "+a"(pf[2]), "+a"(pf[3]), "+a"(pf[4]), "+a"(pf[5]), "+a"(pf[6]),
                 "+a"(pf[7]), "+a"(pf[8]), "+a"(pf[9]), "+a"(pf[10])
               : "n"(N) : "memory");
}
template <int OFF>
__device__ __forceinline__ void st16(unsigned addr, const u32x4& v) {
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "a"(v), "i"(OFF) : "memory");
}
__device__ __forceinline__ void st8(unsigned addr, const u32x2& v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "a"(v) : "memory");
}
// chunk U of the lane (tile bytes o = 16(l + 64U) .. o + 15) into the padded rows: each 8-byte half
// lies in one row (2F ≡ 0 mod 8); row = o / 2F by a multiply-high (mrow = ⌈2^32 / 2F⌉, exact for
// o < 2^16), LDS byte = o + pad·row
template <int U>
__device__ __forceinline__ void stage_x(unsigned base, const u32x4* pf, int l, int nch, unsigned mrow,
                                        unsigned pad) {
  if (l + 64 * U < nch) {
    const unsigned o = 16u * (unsigned)(l + 64 * U);
    st8(base + o + pad * __umulhi(o, mrow), u32x2{pf[U][0], pf[U][1]});
    st8(base + o + 8u + pad * __umulhi(o + 8u, mrow), u32x2{pf[U][2], pf[U][3]});
  }
  if constexpr (U + 1 < PFX) stage_x<U + 1>(base, pf, l, nch, mrow, pad);
}
}  // namespace bw


// ------------------------------------------------------------------------------------------------
// The sample-lane pass: the IOP grid's headline shape (F = 81, k = 4, fp32 X and W), full tiles.
//
// mu_pass_kernel spends most of its issue slots and LDS cycles on moving data between lane
// layouts (Hᵀ re-read by every sample quarter, quad shuffles of the partial dot products, and an
// A phase that re-reads the whole X tile from LDS with 85 of 128 lanes busy).  Here lane = sample
// in every phase that touches X, so each X element is read from LDS exactly once and stays in a
// register from the dot product to the accumulation:
//
//   phase 1  wave w owns features [21w, 21w+21) (wave 3: 63..80 plus three zero Hᵀ rows), lane s
//            owns sample s of the 64-sample tile: xv[c] = x[s][21w+c] (conflict-free ds_read_b32,
//            row stride 81 is odd), partial num_w[s][j] = Σ_c xv[c]·Ht[21w+c][j] as fp32 chains of
//            7 folded into fp64 (the precision note above phase12), written to LDS (32 B per lane).
//   phase 2  lane (s = 16w + lane/4, j = lane%4): num = (P0+P1)+(P2+P3) (the same fp64 sum order as
//            phase12's quad shuffles), den = Σ_m w[s][m]·HHt[j][m] (+l1)(+l2·w), eps32, w' = w·num/den
//            in fp64 (SK:526-631) -> W in HBM (64 consecutive floats per wave) and LDS.
//   phase 3  lane = sample again: acc[c][j] += w'[s][j]·xv[c] on the registers of phase 1; wave 3
//            swaps its three padding columns for the W' columns 81..83, and the last column of
//            B = W'ᵀW' comes from its symmetry (B[j][3] = B[3][j]) plus one Σ w'3² register.
//            (SK:639-640 for the updated W.)
//
// A tile therefore costs per wave 21 x reads + 21 broadcast Hᵀ reads + 6 small LDS accesses,
// about 200 VALU and 2 barriers.  The 21×4 (+1) fp32 accumulators of a lane (fp32 chains of one sample
// per tile over the workgroup's tiles) are tree-summed across the wave with DPP at the end of the
// launch and written as ONE fp64 partial row [k][F+k] per workgroup, like mu_pass_kernel.
// Registers: acc 85 + xv 21 + the next tile's 16-byte prefetch 24 -> three waves per SIMD.
// ------------------------------------------------------------------------------------------------
namespace sl {
constexpr int F = 81, K = 4, V = F + K;
constexpr int NF = 21;                     // features per wave in phase 1 (4 × 21 = 84 ≥ 81)
constexpr int NC = 21;                     // accumulator columns per wave (wave 3: 18 X + W'0..2)
constexpr int NR = NC * 4 + 1;             // row-sum values per wave (+ wave 3's Σ w'3²)
constexpr int XB = TS * F * 4;             // 20736 bytes of X per tile
constexpr int WB = TS * K * 4;             // 1024 bytes of W per tile
constexpr int NXC = XB / 16;               // 1296 X chunks
constexpr int NCH = (XB + WB) / 16;        // 1360 chunks per tile
constexpr int PFN = (NCH + NT - 1) / NT;   // 6 chunks per thread
constexpr int RED = NWAVE * 4 * NR * 4;    // end-of-launch row sums: [wave][row][NR] floats
// LDS carve (bytes)
constexpr int L_X = 0;                                      // X tile + 16 zero bytes; later RED
constexpr int L_W = ((XB + 16 > RED ? XB + 16 : RED) + 15) / 16 * 16;  // W tiles, double-buffered
constexpr int L_P = L_W + 2 * WB;                           // phase-1 partials [wave][s][j] fp64
constexpr int L_WN = L_P + NWAVE * TS * K * 8;              // new W tile [s][j] fp32
constexpr int L_HT = L_WN + TS * K * 4;                     // Hᵀ [84][4] fp32 (rows >= 81 zero)
constexpr int L_HHT = L_HT + NWAVE * NF * K * 4;            // HHᵀ [4][4] fp64
constexpr int L_TOTAL = L_HHT + K * K * 8;
static_assert(PFN == 6 && NCH - (PFN - 1) * NT == 80, "prefetch layout assumes 1360 chunks");

template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
  const int m = __builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true);
  return v + __int_as_float(m);
}

// 16-byte chunk i of this thread for tile `tile`: X chunk (t + 256 i), or for i = 5 and t < 80 the
// tail of X (t < 16) / the W tile (16 <= t < 80); threads t >= 80 re-read X chunk t (not stored).
// LOADW = false (W resident in LDS): the W slots re-read X chunk t as well.
#ifdef CNMF_X_PLAIN  // diagnostic build: default-policy X loads instead of non-temporal ones
#define SL_XLOAD(p) (*(p))
#else
#define SL_XLOAD(p) __builtin_nontemporal_load(p)
#endif
template <bool LOADW = true>
__device__ __forceinline__ void sl_prefetch(u32x4 (&pf)[PFN], const unsigned char* __restrict__ X,
                                            const unsigned char* __restrict__ W, int64_t tile, int t) {
#ifdef CNMF_DIAG_L2  // diagnostic build: every tile reads one of 64 L2-resident tiles (compute floor)
  const unsigned char* xs = X + (size_t)(tile & 63) * XB + 16 * t;
#else
  const unsigned char* xs = X + (size_t)tile * XB + 16 * t;
#endif
#pragma unroll
  for (int i = 0; i < PFN - 1; ++i)
    pf[i] = SL_XLOAD(reinterpret_cast<const u32x4*>(xs + 4096 * i));
  const unsigned char* last = t < 16 ? xs + 4096 * (PFN - 1)
                                     : ((LOADW && t < 80) ? W + (size_t)tile * WB + 16 * (t - 16) : xs);
  pf[PFN - 1] = SL_XLOAD(reinterpret_cast<const u32x4*>(last));
}

template <bool STAGEW = true>
__device__ __forceinline__ void sl_stage(unsigned char* smem, int wpar, const u32x4 (&pf)[PFN], int t) {
#pragma unroll
  for (int i = 0; i < PFN - 1; ++i)
    *reinterpret_cast<u32x4*>(smem + L_X + 16 * t + 4096 * i) = pf[i];
  if (t < (STAGEW ? 80 : 16)) {
    unsigned char* dst = t < 16 ? smem + L_X + 16 * t + 4096 * (PFN - 1)
                                : smem + L_W + wpar * WB + 16 * (t - 16);
    *reinterpret_cast<u32x4*>(dst) = pf[PFN - 1];
  }
}

// the floating-tile (DYN) forms.  The same instruction sequence for every tile, static or floating
// (runtime branches around the loads cost the compiler's waitcnt precision: ~0.6 µs per tile): X as in
// sl_prefetch<false>, plus one 16-byte sc1 load per lane (two 8-byte agent-scope loads) that fetches
// the tile's W when it floats (lanes 16..79) and otherwise re-reads the lane's first X chunk.
// sc1 because a floating tile's W was stored sc1 by whichever workgroup (any XCD) processed it in the
// previous iteration (MI355X_MICROARCH.md valid forms: sc1 stores, vmcnt(0), ticket, flag, sc1 loads).
__device__ __forceinline__ void sl_prefetch_w(uint64_t (&pw)[2], const unsigned char* __restrict__ X,
                                              const unsigned char* __restrict__ W, int64_t tile, bool flt, int t) {
  // static tile: the lane's own first X chunk of the tile (just loaded by sl_prefetch, spread over
  // the channels like X; a fixed line set shared by every workgroup serialised on one channel)
  const unsigned char* src = flt ? W + (size_t)tile * WB + 16 * ((t - 16) & 63) : X + (size_t)tile * XB + 16 * t;
  uint64_t* l = reinterpret_cast<uint64_t*>(const_cast<unsigned char*>(src));
  pw[0] = __hip_atomic_load(l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  pw[1] = __hip_atomic_load(l + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void sl_stage_w(unsigned char* smem, int wpar, const uint64_t (&pw)[2], int t) {
  if (t >= 16 && t < 80)  // a static tile's lanes write the unused W slot (never read)
    *reinterpret_cast<u32x4*>(smem + L_W + wpar * WB + 16 * (t - 16)) =
        u32x4{(unsigned)pw[0], (unsigned)(pw[0] >> 32), (unsigned)pw[1], (unsigned)(pw[1] >> 32)};
}

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes are done
  __builtin_amdgcn_s_barrier();
}
}  // namespace sl

namespace sl {
// ---- the three phases of one tile (shared by mu_pass_sl_kernel and mu_iter_sl_kernel)

// phase 1: lane = sample, wave = 21 features: xv[] <- x[lane][21w..21w+20], partial num -> sP
__device__ __forceinline__ void phase1(unsigned char* smem, float (&xv)[NC], int wave, int lane) {
  const float* sX = reinterpret_cast<const float*>(smem + L_X);
  const float* sHt = reinterpret_cast<const float*>(smem + L_HT);
  double* sP = reinterpret_cast<double*>(smem + L_P);
  const int fbase = NF * wave;
  const float* xr = sX + lane * F + fbase;
#pragma unroll
  for (int c = 0; c < NF; ++c) xv[c] = xr[c];
  double p[K] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c0 = 0; c0 < NF; c0 += 7) {
    float pc[K] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = c0; c < c0 + 7; ++c) {
      const float4 h = *reinterpret_cast<const float4*>(sHt + (fbase + c) * K);
      pc[0] = fmaf(xv[c], h.x, pc[0]);
      pc[1] = fmaf(xv[c], h.y, pc[1]);
      pc[2] = fmaf(xv[c], h.z, pc[2]);
      pc[3] = fmaf(xv[c], h.w, pc[3]);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) p[j] += (double)pc[j];
  }
  double* pw = sP + ((size_t)wave * TS + lane) * K;
  *reinterpret_cast<double2*>(pw) = make_double2(p[0], p[1]);
  *reinterpret_cast<double2*>(pw + 2) = make_double2(p[2], p[3]);
}

// phase 2: lane = (sample 16w + lane/4, component lane%4): the MU update of w[s][j] in fp64
// wres (W resident in LDS, mu_iter_sl_kernel<…, true>): this tile's W [64][4] is read from and
// the new W written back to LDS; otherwise the staged tile is read and the new W stored to HBM.
__device__ __forceinline__ void phase2(unsigned char* smem, float* __restrict__ W, int64_t tile, int wpar,
                                       int wave, int lane, double l1, double l2, float* wres = nullptr,
                                       bool active = true, bool sc1w = false) {
  const double* sP = reinterpret_cast<const double*>(smem + L_P);
  const double* sHHt = reinterpret_cast<const double*>(smem + L_HHT);
  float* sWn = reinterpret_cast<float*>(smem + L_WN);
  const int s = 16 * wave + (lane >> 2);
  const int j = lane & 3;
  const double num = (sP[(0 * TS + s) * K + j] + sP[(1 * TS + s) * K + j]) +
                     (sP[(2 * TS + s) * K + j] + sP[(3 * TS + s) * K + j]);
  const float* sWo = wres ? wres : reinterpret_cast<const float*>(smem + L_W + wpar * WB);
  const float4 wv = *reinterpret_cast<const float4*>(sWo + s * K);
  const double wold = (double)sWo[s * K + j];
  const double* hr = sHHt + j * K;
  double den = 0.0;
  den = fma((double)wv.x, hr[0], den);
  den = fma((double)wv.y, hr[1], den);
  den = fma((double)wv.z, hr[2], den);
  den = fma((double)wv.w, hr[3], den);
  if (l1 > 0.0) den += l1;              // SK:616-617
  if (l2 > 0.0) den = den + l2 * wold;  // SK:618-619
  if (den == 0.0) den = EPS32;          // SK:620
  const float wn = (float)(wold * (num / den));  // SK:622-629
  // inactive: a padding step of the team with one tile fewer (mu_iter_sl_kernel<…, 2>): nothing
  // is stored and w' = 0 makes phase 3 add nothing
  if (active) {
    if (wres) wres[s * K + j] = wn;  // the quad's float4 read above precedes this store (data dependence)
    if (sc1w)  // a floating tile: another workgroup (any XCD) reads this W next iteration
      __hip_atomic_store(W + ((size_t)tile * TS + s) * K + j, wn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (!wres)
      W[((size_t)tile * TS + s) * K + j] = wn;
  }
  sWn[s * K + j] = active ? wn : 0.f;
}

// phase 3: lane = sample; acc += w'ᵀ·[x | w'] on the registers of phase 1 (SK:639-640)
__device__ __forceinline__ void phase3(const unsigned char* smem, float (&xv)[NC], float (&acc)[NC][K],
                                       float& acc33, int wave, int lane) {
  const float* sWn = reinterpret_cast<const float*>(smem + L_WN);
  const float4 w4 = *reinterpret_cast<const float4*>(sWn + lane * K);
  if (wave == NWAVE - 1) {  // columns 81..83 of [X | W'] (its xv[18..20] were Hᵀ padding)
    xv[NC - 3] = w4.x;
    xv[NC - 2] = w4.y;
    xv[NC - 1] = w4.z;
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    acc[c][0] = fmaf(w4.x, xv[c], acc[c][0]);
    acc[c][1] = fmaf(w4.y, xv[c], acc[c][1]);
    acc[c][2] = fmaf(w4.z, xv[c], acc[c][2]);
    acc[c][3] = fmaf(w4.w, xv[c], acc[c][3]);
  }
  acc33 = fmaf(w4.w, w4.w, acc33);
}

// The workgroup's accumulators -> its fp64 partial row [K][V]: a DPP tree over each 16-lane row,
// the 4 row sums of each wave through LDS (`red`, NWAVE*4*NR floats), the 4 waves summed in fp64.
// SC1: store the row write-through (an in-launch hand-off, MI355X_MICROARCH.md valid-forms table).
// TEAMS = 2 (the two 4-wave teams of an 8-wave workgroup, mu_iter_sl_kernel<…, 2>): each team
// reduces into its own scratch `red`; after the barrier the 512 threads (tid) combine team 0's and
// team 1's (`red0`, `red1`) wave sums in a fixed order into the workgroup's one row.
template <bool SC1, int TEAMS = 1>
__device__ __forceinline__ void flush_acc(float* red, float (&acc)[NC][K], float& acc33, double* prow,
                                          int wave, int lane, int t, const float* red0 = nullptr,
                                          const float* red1 = nullptr, int tid = 0) {
  float* myred = red + (wave * 4 + (lane >> 4)) * NR;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < K; ++j) {
      float r = acc[c][j];
      r = dpp_add<0xB1>(r);   // quad_perm [1,0,3,2]
      r = dpp_add<0x4E>(r);   // quad_perm [2,3,0,1]
      r = dpp_add<0x141>(r);  // row_half_mirror
      r = dpp_add<0x140>(r);  // row_mirror: every lane holds its row's sum
      if ((lane & 15) == 0) myred[c * K + j] = r;
    }
  {
    float r = acc33;
    r = dpp_add<0xB1>(r);
    r = dpp_add<0x4E>(r);
    r = dpp_add<0x141>(r);
    r = dpp_add<0x140>(r);
    if ((lane & 15) == 0) myred[NC * K] = r;
  }
  lds_barrier();
  for (int e = TEAMS == 1 ? t : tid; e < K * V; e += NT * TEAMS) {
    const int j = e / V;
    const int v = e - j * V;
    const int w = v < 3 * NF ? v / NF : 3;
    int idx;  // position inside wave w's row sums
    if (v < V - 1) idx = (v - NF * w) * K + j;
    else idx = j < K - 1 ? (NC - 3 + j) * K + (K - 1) : NC * K;  // column 84 = B[.][3] = B[3][.]
    const float* rr = (TEAMS == 1 ? red : red0) + (w * 4) * NR + idx;
    double val = ((double)rr[0] + (double)rr[NR]) + ((double)rr[2 * NR] + (double)rr[3 * NR]);
    if (TEAMS == 2) {
      const float* r1 = red1 + (w * 4) * NR + idx;
      val += ((double)r1[0] + (double)r1[NR]) + ((double)r1[2 * NR] + (double)r1[3 * NR]);
    }
    if (SC1)
      __hip_atomic_store(prow + e, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      prow[e] = val;
  }
}
}  // namespace sl

// ------------------------------------------------------------------------------------------------
// The constrained-ALS W-step on the sample-lane layout (cfg5: fp32 X, F = 81, k = 4, full tiles):
// phase 1 forms c = Hx in fp64 (lane = sample, wave = 21 features, Hᵀ in fp64 in LDS; the solve
// amplifies errors by cond(Q), so no fp32 chains here), phase 2 is the exact FCLS of phase12's
// ALS branch (lane = (sample, component): the 16 passive sets, 4 per lane, least objective by quad
// shuffles; oracle/als_ref.py), phase 3 the sl accumulation of [WᵀX | WᵀW] (SK:639-640 form).
// ------------------------------------------------------------------------------------------------
namespace sl {
constexpr int L_HT64 = (L_TOTAL + 15) / 16 * 16;      // Hᵀ fp64 [84][4] (rows >= 81 zero)
constexpr int L_TAB = L_HT64 + NWAVE * NF * K * 8;     // passive-set table (ALS_TAB doubles)
constexpr int L_ALS_TOTAL = L_TAB + ALS_TAB * 8;
}  // namespace sl

__global__ __launch_bounds__(NT, 2) void als_pass_sl_kernel(const float* __restrict__ X,
                                                           float* __restrict__ W,
                                                           const double* __restrict__ Ht,
                                                           const double* __restrict__ table,
                                                           double* __restrict__ partials,
                                                           int64_t n_tiles, double delta2,
                                                           int64_t n_rows_out) {
  using namespace sl;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const unsigned char* Xb = reinterpret_cast<const unsigned char*>(X);
  const unsigned char* Wb = reinterpret_cast<const unsigned char*>(W);
  double* sHt = reinterpret_cast<double*>(smem + L_HT64);
  double* sTab = reinterpret_cast<double*>(smem + L_TAB);
  double* sP = reinterpret_cast<double*>(smem + L_P);
  float* sWn = reinterpret_cast<float*>(smem + L_WN);

  for (int e = t; e < NWAVE * NF * K; e += NT) sHt[e] = e < F * K ? Ht[e] : 0.0;
  for (int e = t; e < ALS_TAB; e += NT) sTab[e] = table[e];
  if (t < 4) reinterpret_cast<float*>(smem + L_X + XB)[t] = 0.f;

  float acc[NC][K];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < K; ++j) acc[c][j] = 0.f;
  float acc33 = 0.f;

  const int64_t G = gridDim.x;
  int64_t tile = blockIdx.x;
  u32x4 pf[PFN];
  sl_prefetch(pf, Xb, Wb, tile, t);
  sl_stage(smem, 0, pf, t);
  if (tile + G < n_tiles) sl_prefetch(pf, Xb, Wb, tile + G, t);
  lds_barrier();

  int wpar = 0;
  for (; tile < n_tiles; tile += G, wpar ^= 1) {
    // ---- phase 1: c partials in fp64 (lane = sample, wave = 21 features)
    float xv[NC];
    {
      const float* xr = reinterpret_cast<const float*>(smem + L_X) + lane * F + NF * wave;
#pragma unroll
      for (int c = 0; c < NF; ++c) xv[c] = xr[c];
      double p[K] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int c = 0; c < NF; ++c) {
        const double* h = sHt + (NF * wave + c) * K;
        const double2 h01 = *reinterpret_cast<const double2*>(h);
        const double2 h23 = *reinterpret_cast<const double2*>(h + 2);
        const double x = (double)xv[c];
        p[0] = fma(x, h01.x, p[0]);
        p[1] = fma(x, h01.y, p[1]);
        p[2] = fma(x, h23.x, p[2]);
        p[3] = fma(x, h23.y, p[3]);
      }
      double* pw = sP + ((size_t)wave * TS + lane) * K;
      *reinterpret_cast<double2*>(pw) = make_double2(p[0], p[1]);
      *reinterpret_cast<double2*>(pw + 2) = make_double2(p[2], p[3]);
    }
    lds_barrier();  // A
    // ---- phase 2: exact FCLS per sample, lane = (sample 16w + lane/4, component lane%4)
    {
      const int s = 16 * wave + (lane >> 2);
      const int qtr = lane & 3;
      double c[K];
#pragma unroll
      for (int j = 0; j < K; ++j)
        c[j] = ((sP[(0 * TS + s) * K + j] + sP[(1 * TS + s) * K + j]) +
                (sP[(2 * TS + s) * K + j] + sP[(3 * TS + s) * K + j])) + delta2;
      double bestf = 1.0;
      int bestm = 16;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int m = qtr + 4 * u;
        const double* T = sTab + m * 16;
        bool feas = sTab[256 + m] != 0.0;
        double f = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double v = 0.0;
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) v = fma(T[r * 4 + cc], c[cc], v);
          feas = feas && v >= 0.0;
          f = fma(c[r], v, f);
        }
        f *= -0.5;
        if (feas && (f < bestf || (f == bestf && m < bestm))) {
          bestf = f;
          bestm = m;
        }
      }
#pragma unroll
      for (int off = 1; off <= 2; off <<= 1) {
        const double of = __shfl_xor(bestf, off);
        const int om = __shfl_xor(bestm, off);
        if (of < bestf || (of == bestf && om < bestm)) {
          bestf = of;
          bestm = om;
        }
      }
      const double* T = sTab + min(bestm, 15) * 16;
      double wn64 = 0.0;
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) wn64 = fma(T[qtr * 4 + cc], c[cc], wn64);
      const float wn = (float)fmax(wn64, 0.0);
      W[((size_t)tile * TS + s) * K + qtr] = wn;
      sWn[s * K + qtr] = wn;
    }
    if (tile + G < n_tiles) {
      sl_stage(smem, wpar ^ 1, pf, t);
      if (tile + 2 * G < n_tiles) sl_prefetch(pf, Xb, Wb, tile + 2 * G, t);
    }
    lds_barrier();  // B
    phase3(smem, xv, acc, acc33, wave, lane);
  }
  lds_barrier();
  flush_acc<false>(reinterpret_cast<float*>(smem + L_X), acc, acc33,
                   partials + (size_t)blockIdx.x * (K * V), wave, lane, t);
  // partial rows beyond this grid (the caller's row count is the sl grid) are zero
  for (int64_t r = blockIdx.x + G; r < n_rows_out; r += G)
    for (int e = t; e < K * V; e += NT) partials[(size_t)r * (K * V) + e] = 0.0;
}

__global__ __launch_bounds__(NT, 3) void mu_pass_sl_kernel(const float* __restrict__ X,
                                                          float* __restrict__ W,
                                                          const double* __restrict__ Ht,
                                                          const double* __restrict__ HHt,
                                                          double* __restrict__ partials,
                                                          int64_t n_tiles, double l1, double l2) {
  using namespace sl;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const unsigned char* Xb = reinterpret_cast<const unsigned char*>(X);
  const unsigned char* Wb = reinterpret_cast<const unsigned char*>(W);
  float* sHt = reinterpret_cast<float*>(smem + L_HT);
  double* sHHt = reinterpret_cast<double*>(smem + L_HHT);
  double* sP = reinterpret_cast<double*>(smem + L_P);
  float* sWn = reinterpret_cast<float*>(smem + L_WN);

  for (int e = t; e < NWAVE * NF * K; e += NT) sHt[e] = e < F * K ? (float)Ht[e] : 0.f;
  if (t < K * K) sHHt[t] = HHt[t];
  if (t < 4) reinterpret_cast<float*>(smem + L_X + XB)[t] = 0.f;

  float acc[NC][K];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < K; ++j) acc[c][j] = 0.f;
  float acc33 = 0.f;

  const int64_t G = gridDim.x;
  int64_t tile = blockIdx.x;
  u32x4 pf[PFN];
  // prologue: tile `tile` -> LDS, tile + G -> registers
  sl_prefetch(pf, Xb, Wb, tile, t);
  sl_stage(smem, 0, pf, t);
  if (tile + G < n_tiles) sl_prefetch(pf, Xb, Wb, tile + G, t);
  lds_barrier();

  const float* sX = reinterpret_cast<const float*>(smem + L_X);
  const int fbase = NF * wave;
  int wpar = 0;
  for (; tile < n_tiles; tile += G, wpar ^= 1) {
    // ---- phase 1: lane = sample, wave = 21 features
    float xv[NC];
    {
      const float* xr = sX + lane * F + fbase;
#pragma unroll
      for (int c = 0; c < NF; ++c) xv[c] = xr[c];
      double p[K] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int c0 = 0; c0 < NF; c0 += 7) {
        float pc[K] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = c0; c < c0 + 7; ++c) {
          const float4 h = *reinterpret_cast<const float4*>(sHt + (fbase + c) * K);
          pc[0] = fmaf(xv[c], h.x, pc[0]);
          pc[1] = fmaf(xv[c], h.y, pc[1]);
          pc[2] = fmaf(xv[c], h.z, pc[2]);
          pc[3] = fmaf(xv[c], h.w, pc[3]);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) p[j] += (double)pc[j];
      }
      double* pw = sP + ((size_t)wave * TS + lane) * K;
      *reinterpret_cast<double2*>(pw) = make_double2(p[0], p[1]);
      *reinterpret_cast<double2*>(pw + 2) = make_double2(p[2], p[3]);
    }
    lds_barrier();  // A: every wave is done reading this X tile and has written its partials

    // ---- phase 2: lane = (sample 16w + lane/4, component lane%4)
    {
      const int s = 16 * wave + (lane >> 2);
      const int j = lane & 3;
      const double num = (sP[(0 * TS + s) * K + j] + sP[(1 * TS + s) * K + j]) +
                         (sP[(2 * TS + s) * K + j] + sP[(3 * TS + s) * K + j]);
      const float* sWo = reinterpret_cast<const float*>(smem + L_W + wpar * WB);
      const float4 wv = *reinterpret_cast<const float4*>(sWo + s * K);
      const double wold = (double)sWo[s * K + j];
      const double* hr = sHHt + j * K;
      double den = 0.0;
      den = fma((double)wv.x, hr[0], den);
      den = fma((double)wv.y, hr[1], den);
      den = fma((double)wv.z, hr[2], den);
      den = fma((double)wv.w, hr[3], den);
      if (l1 > 0.0) den += l1;              // SK:616-617
      if (l2 > 0.0) den = den + l2 * wold;  // SK:618-619
      if (den == 0.0) den = EPS32;          // SK:620
      const float wn = (float)(wold * (num / den));  // SK:622-629
      W[((size_t)tile * TS + s) * K + j] = wn;
      sWn[s * K + j] = wn;
    }
    // ---- stage the next tile (X region is free since barrier A) and prefetch the one after
    if (tile + G < n_tiles) {
      sl_stage(smem, wpar ^ 1, pf, t);
      if (tile + 2 * G < n_tiles) sl_prefetch(pf, Xb, Wb, tile + 2 * G, t);
    }
    lds_barrier();  // B: W' tile and the next X tile are visible

    // ---- phase 3: lane = sample; acc += w'ᵀ·[x | w'] on the registers of phase 1
    {
      const float4 w4 = *reinterpret_cast<const float4*>(sWn + lane * K);
      if (wave == NWAVE - 1) {  // columns 81..83 of [X | W'] (its xv[18..20] were Hᵀ padding)
        xv[NC - 3] = w4.x;
        xv[NC - 2] = w4.y;
        xv[NC - 1] = w4.z;
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        acc[c][0] = fmaf(w4.x, xv[c], acc[c][0]);
        acc[c][1] = fmaf(w4.y, xv[c], acc[c][1]);
        acc[c][2] = fmaf(w4.z, xv[c], acc[c][2]);
        acc[c][3] = fmaf(w4.w, xv[c], acc[c][3]);
      }
      acc33 = fmaf(w4.w, w4.w, acc33);
    }
  }

  // ---- end of launch: DPP tree over each 16-lane row, row sums via LDS, fp64 partial row
  lds_barrier();  // the X region becomes the row-sum scratch
  float* red = reinterpret_cast<float*>(smem + L_X);
  float* myred = red + (wave * 4 + (lane >> 4)) * NR;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < K; ++j) {
      float r = acc[c][j];
      r = dpp_add<0xB1>(r);   // quad_perm [1,0,3,2]
      r = dpp_add<0x4E>(r);   // quad_perm [2,3,0,1]
      r = dpp_add<0x141>(r);  // row_half_mirror
      r = dpp_add<0x140>(r);  // row_mirror: every lane holds its row's sum
      if ((lane & 15) == 0) myred[c * K + j] = r;
    }
  {
    float r = acc33;
    r = dpp_add<0xB1>(r);
    r = dpp_add<0x4E>(r);
    r = dpp_add<0x141>(r);
    r = dpp_add<0x140>(r);
    if ((lane & 15) == 0) myred[NC * K] = r;
  }
  lds_barrier();
  double* prow = partials + (size_t)blockIdx.x * (K * V);
  for (int e = t; e < K * V; e += NT) {
    const int j = e / V;
    const int v = e - j * V;
    const int w = v < 3 * NF ? v / NF : 3;
    int idx;  // position inside wave w's row sums
    if (v < V - 1) idx = (v - NF * w) * K + j;
    else idx = j < K - 1 ? (NC - 3 + j) * K + (K - 1) : NC * K;  // column 84 = B[.][3] = B[3][.]
    const float* rr = red + (w * 4) * NR + idx;
    prow[e] = ((double)rr[0] + (double)rr[NR]) + ((double)rr[2 * NR] + (double)rr[3 * NR]);
  }
}

// ------------------------------------------------------------------------------------------------
// Basis update (one workgroup): the k×F epilogue, all in fp64.
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline size_t update_mfma_lds_doubles(int F);
__host__ __device__ inline size_t update_lds_doubles(int F, int k, int KP) {
  if (KP >= 8) return update_mfma_lds_doubles(F);
  return 2 * (size_t)k * F + (size_t)k * k + (size_t)KP * KP + 2 * (RED_NT / 64);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// The basis update for KP >= 8 on v_mfma_f64_16x16x4_f64 (exact fp64; C/D layout row = g + 4·reg,
// col = lane & 15; A/B as the f32 16x16x4 form): den = (WᵀW)·H per 16-feature block and HHᵀ = H·Hᵀ
// with the 4 waves splitting K = F, their partials summed in fixed order.  H is staged in LDS
// ([16][F16], zero rows >= k and columns >= F) and updated in place; AB comes from a previous
// launch (the reduction), so plain loads see it.
// Per element the same arithmetic as basis_update_block (den a k-ordered fma chain, SK:634-728).
__host__ __device__ inline int f16pad(int F) { return (F + 15) / 16 * 16; }
__host__ __device__ inline size_t update_mfma_lds_doubles(int F) {
  return 16 * (size_t)f16pad(F) + 16 * 16 + 4 * 64 * 4 + 2 * 4;
}

__device__ void basis_update_mfma(const double* AB, double* H64, double* Ht, double* HHt, int F, int k,
                                  int KP, double l1, double l2, int do_update, double* stats, double* lds) {
  typedef double f64x4v __attribute__((ext_vector_type(4)));
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int V = F + k;
  const int FP = f16pad(F);
  const int NB = FP / 16;
  double* sH = lds;                   // [16][FP]
  double* sB = sH + 16 * FP;          // [16][16], zero beyond k
  double* red = sB + 256;             // [4 waves][64 lanes][4]
  double* sR = red + 4 * 64 * 4;      // [2][4]
  const bool upd = do_update && AB != nullptr;
  // H into LDS with 8 loads per thread in flight (one load per trip of a runtime loop waited for each
  // one in turn: 19 dependent global round trips at F = 300 were most of this kernel's 23 µs)
  constexpr int UB = 8;
  for (int e0 = t; e0 < 16 * FP; e0 += RED_NT * UB) {
    double v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int e = e0 + u * RED_NT;
      const int j = e / FP, f = e - j * FP;
      const bool ok = e < 16 * FP && j < k && f < F;
      const double x = H64[ok ? j * F + f : 0];
      v[u] = ok ? x : 0.0;
    }
#pragma unroll
    for (int u = 0; u < UB; ++u)
      if (e0 + u * RED_NT < 16 * FP) sH[e0 + u * RED_NT] = v[u];
  }
  for (int e = t; e < 256; e += RED_NT) {
    const int j = e >> 4, m = e & 15;
    sB[e] = (upd && j < k && m < k) ? AB[j * V + F + m] : 0.0;
  }
  __syncthreads();
  if (upd) {
    constexpr int NBL = 8;  // F <= 512
    double hn[NBL][4];
    double bfr[4];
    // this lane's numerators (WᵀX)[j][f], all loads in flight together
    double nm[NBL][4];
#pragma unroll
    for (int i = 0; i < NBL; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = g + 4 * r, f = 16 * (wave + 4 * i) + li;
        const bool ok = wave + 4 * i < NB && j < k && f < F;
        const double x = AB[ok ? j * V + f : 0];
        nm[i][r] = ok ? x : 0.0;
      }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) bfr[kk] = sB[li * 16 + 4 * kk + g];  // A[j = li][m = 4kk + g]
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
      const int nb = wave + 4 * i;
      if (nb >= NB) break;
      const int f = 16 * nb + li;
      f64x4v den = f64x4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        den = __builtin_amdgcn_mfma_f64_16x16x4f64(bfr[kk], sH[(4 * kk + g) * FP + f], den, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = g + 4 * r;
        double h = sH[j * FP + f];
        if (j < k && f < F) {
          const double num = nm[i][r];
          double d = den[r];
          if (l1 > 0.0) d += l1;                                // SK:702-703
          if (l2 > 0.0) d = d + l2 * h;                         // SK:704-705
          if (d == 0.0) d = EPS32;                              // SK:706
          h = h * (num / d);                                    // SK:722-726
        }
        hn[i][r] = h;
      }
    }
    __syncthreads();  // every old H read is done before sH is overwritten
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
      const int nb = wave + 4 * i;
      if (nb >= NB) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) sH[(g + 4 * r) * FP + 16 * nb + li] = hn[i][r];
    }
    __syncthreads();
  }
  for (int e = t; e < k * F; e += RED_NT) H64[e] = sH[(e / F) * FP + (e % F)];
  for (int e = t; e < F * KP; e += RED_NT) {
    const int f = e / KP, j = e - f * KP;
    Ht[e] = j < k ? sH[j * FP + f] : 0.0;
  }
  // HHᵀ: K = F in steps of 4 features, step kk on wave kk % 4; A[j = li][f] = B[f][m = li] = H[li][f]
  f64x4v hh = f64x4v{0.0, 0.0, 0.0, 0.0};
  for (int kk = wave; 4 * kk < FP; kk += 4) {
    const double v = sH[li * FP + 4 * kk + g];
    hh = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, hh, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[(wave * 64 + lane) * 4 + r] = hh[r];
  __syncthreads();
  {
    const int l = t & 63, r = t >> 6;  // entry (j = (l >> 4) + 4r, m = l & 15)
    const int j = (l >> 4) + 4 * r, m = l & 15;
    const double v = ((red[(0 * 64 + l) * 4 + r] + red[(1 * 64 + l) * 4 + r]) + red[(2 * 64 + l) * 4 + r]) +
                     red[(3 * 64 + l) * 4 + r];
    if (j < KP && m < KP) HHt[j * KP + m] = v;
    if (stats && upd) {
      double a = 0.0, b = 0.0;
      for (int e = t; e < k * F; e += RED_NT)
        a = fma(AB[(e / F) * V + (e % F)], sH[(e / F) * FP + (e % F)], a);
      if (j < k && m < k) b = sB[j * 16 + m] * v;
      a = wave_sum(a);
      b = wave_sum(b);
      if (lane == 0) {
        sR[wave] = a;
        sR[4 + wave] = b;
      }
      __syncthreads();
      if (t == 0) {
        stats[0] = ((sR[0] + sR[1]) + sR[2]) + sR[3];
        stats[1] = ((sR[4] + sR[5]) + sR[6]) + sR[7];
      }
    }
  }
}

__device__ void basis_update_block(const double* AB, double* H64, double* Ht, double* HHt, int F,
                                   int k, int KP, double l1, double l2, int do_update, double* stats,
                                   double* lds);

// the KP = 4 basis update (one wave per HHᵀ entry; the arithmetic sl_update_basis repeats)
__device__ void basis_update_small(const double* AB, double* H64, double* Ht, double* HHt, int F,
                                   int k, int KP, double l1, double l2, int do_update, double* stats,
                                   double* lds) {
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  constexpr int NWV = RED_NT / 64;
  const int V = F + k;
  double* sH = lds;                  // [k][F] new H
  double* sH0 = sH + (size_t)k * F;  // [k][F] old H
  double* sB = sH0 + (size_t)k * F;  // [k][k] WᵀW
  double* sHH = sB + (size_t)k * k;  // [KP][KP] H·Hᵀ
  double* sR = sHH + (size_t)KP * KP;  // [2][NWV]

  const bool have_ab = AB != nullptr;  // NULL when only deriving Ht/HHt from H64 (do_update=0)
  for (int e = t; e < k * F; e += RED_NT) sH0[e] = H64[e];
  if (have_ab)
    for (int e = t; e < k * k; e += RED_NT) sB[e] = AB[(e / k) * V + F + (e % k)];
  __syncthreads();
  for (int e = t; e < k * F; e += RED_NT) {
    const int j = e / F;
    const int f = e - j * F;
    double h = sH0[e];
    if (do_update && have_ab) {
      const double num = AB[j * V + f];                       // (WᵀX)[j][f], SK:639
      double den = 0.0;                                       // ((WᵀW)·H)[j][f], SK:640
      for (int m = 0; m < k; ++m) den = fma(sB[j * k + m], sH0[m * F + f], den);
      if (l1 > 0.0) den += l1;                                // SK:702-703
      if (l2 > 0.0) den = den + l2 * h;                       // SK:704-705
      if (den == 0.0) den = EPS32;                            // SK:706
      h = h * (num / den);                                    // SK:722-726
    }
    sH[e] = h;
  }
  __syncthreads();
  for (int e = t; e < k * F; e += RED_NT) H64[e] = sH[e];
  for (int e = t; e < F * KP; e += RED_NT) {
    const int f = e / KP;
    const int j = e - f * KP;
    Ht[e] = j < k ? sH[j * F + f] : 0.0;
  }
  // HHt[j][m] = Σ_f H[j][f]·H[m][f]: one wave per entry, lanes over f, fixed-order shuffle tree
  // (the arithmetic sl_derive_basis repeats; KP >= 8 takes basis_update_mfma)
  {
    for (int e = wave; e < KP * KP; e += NWV) {
      const int j = e / KP;
      const int m = e - j * KP;
      double v = 0.0;
      if (j < k && m < k) {
        for (int f = lane; f < F; f += 64) v = fma(sH[j * F + f], sH[m * F + f], v);
        v = wave_sum(v);
      }
      if (lane == 0) {
        sHH[e] = v;
        HHt[e] = v;
      }
    }
  }
  if (stats && have_ab) {
    __syncthreads();
    double a = 0.0, b = 0.0;
    for (int e = t; e < k * F; e += RED_NT) a = fma(AB[(e / F) * V + (e % F)], sH[e], a);
    for (int e = t; e < k * k; e += RED_NT) b = fma(sB[e], sHH[(e / k) * KP + (e % k)], b);
    a = wave_sum(a);
    b = wave_sum(b);
    if (lane == 0) {
      sR[wave] = a;
      sR[NWV + wave] = b;
    }
    __syncthreads();
    if (t == 0) {
      double sa = 0.0, sb = 0.0;
      for (int w = 0; w < NWV; ++w) {
        sa += sR[w];
        sb += sR[NWV + w];
      }
      stats[0] = sa;
      stats[1] = sb;
    }
  }
}

__device__ void basis_update_block(const double* AB, double* H64, double* Ht, double* HHt, int F,
                                   int k, int KP, double l1, double l2, int do_update, double* stats,
                                   double* lds) {
  if (KP >= 8)
    basis_update_mfma(AB, H64, Ht, HHt, F, k, KP, l1, l2, do_update, stats, lds);
  else
    basis_update_small(AB, H64, Ht, HHt, F, k, KP, l1, l2, do_update, stats, lds);
}

// The basis update for KP = 16 (k = 9..16) spread over the 16-feature blocks of H: workgroup nb (one
// wave) updates H[:, 16nb .. 16nb + 15] (den = (WᵀW)·H on v_mfma_f64_16x16x4_f64 in the arithmetic of
// basis_update_mfma, SK:634-728), writes its H64 / Ht columns and its block's HHᵀ partial
// Σ_f h[j][f]·h[m][f] (sc1 stores), takes a ticket, and the last arriver sums the partials in block
// order into HHt (MI355X_MICROARCH.md "valid forms" row 1; one wave per workgroup, so the wave's own
// vmcnt(0) covers every store the ticket signals).  The single-workgroup kernel ran 17.5 µs per cfg4
// iteration on its serial phases (profiles/r03/bfw/bfw1/cfg4_kernel_stats.csv).
__global__ __launch_bounds__(64) void basis_update_split_kernel(const double* __restrict__ AB, double* __restrict__ H64,
                                                                double* __restrict__ Ht, double* __restrict__ HHt,
                                                                int F, int k, double l1, double l2,
                                                                double* __restrict__ scratch, uint32_t* ticket) {
  typedef double f64x4v __attribute__((ext_vector_type(4)));
  __shared__ double sh[16 * 17];
  const int lane = threadIdx.x;
  const int g = lane >> 4, li = lane & 15;
  const int nb = blockIdx.x;
  const int V = F + k;
  const int f = 16 * nb + li;
  const bool fok = f < F;
  double bfr[4], hb[4], num[4], hold[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int m = 4 * kk + g;
    bfr[kk] = (li < k && m < k) ? AB[li * V + F + m] : 0.0;  // (WᵀW)[j = li][m]
    hb[kk] = (m < k && fok) ? H64[m * F + f] : 0.0;           // H[m][f]
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = g + 4 * r;
    const bool ok = j < k && fok;
    num[r] = ok ? AB[j * V + f] : 0.0;   // (WᵀX)[j][f]
    hold[r] = ok ? H64[j * F + f] : 0.0;
  }
  f64x4v den = f64x4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) den = __builtin_amdgcn_mfma_f64_16x16x4f64(bfr[kk], hb[kk], den, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = g + 4 * r;
    double h = hold[r];
    if (j < k && fok) {
      double d = den[r];
      if (l1 > 0.0) d += l1;          // SK:702-703
      if (l2 > 0.0) d = d + l2 * h;   // SK:704-705
      if (d == 0.0) d = EPS32;        // SK:706
      h = h * (num[r] / d);           // SK:722-726
      H64[j * F + f] = h;
    }
    if (fok) Ht[(size_t)f * 16 + j] = j < k ? h : 0.0;
    sh[j * 17 + li] = (j < k && fok) ? h : 0.0;
  }
  // this block's HHᵀ partial: A[j = li][f = 4kk + g] = B[f][m = li] = h[li][4kk + g]
  f64x4v hh = f64x4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const double v = sh[li * 17 + 4 * kk + g];
    hh = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, hh, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)  // P[j = g + 4r][m = li]
    __hip_atomic_store(scratch + ((size_t)nb * 16 + g + 4 * r) * 16 + li, hh[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  if (old != gridDim.x - 1) return;
  // the last arriver: HHᵀ = Σ_nb P_nb in block order (sc1 loads, all of a lane's in flight at once:
  // the host keeps F <= 320, at most 20 blocks)
  constexpr int NBM = 20;
  double x[4][NBM];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int u = 0; u < NBM; ++u)
      x[r][u] = __hip_atomic_load(scratch + (size_t)min(u, (int)gridDim.x - 1) * 256 + (g + 4 * r) * 16 + li,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double v = 0.0;
#pragma unroll
    for (int u = 0; u < NBM; ++u) v += u < (int)gridDim.x ? x[r][u] : 0.0;
    HHt[(g + 4 * r) * 16 + li] = v;
  }
  if (lane == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // at rest
}

__global__ __launch_bounds__(RED_NT) void basis_update_kernel(const double* __restrict__ AB,
                                                              double* __restrict__ H64,
                                                              double* __restrict__ Ht,
                                                              double* __restrict__ HHt, int F, int k,
                                                              int KP, double l1, double l2,
                                                              int do_update, double* stats) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  basis_update_block(AB, H64, Ht, HHt, F, k, KP, l1, l2, do_update, stats,
                     reinterpret_cast<double*>(smem));
}

// ------------------------------------------------------------------------------------------------
// The persistent multi-iteration kernel for the headline shape (F = 81, k = 4, fp32, full tiles):
// n_iter complete MU iterations (SK:831-870 for a tol == 0 stretch) in ONE launch.
//
// Each workgroup keeps the SAME tiles every iteration (static round-robin) and runs the sample-lane
// tile pipeline of mu_pass_sl_kernel over them.  At the end of an iteration its fp64 partial row
// [K][V] is published write-through (sc1) and the cross-block reduction runs in-launch:
//   * groups of <= 16 workgroups (g = block % NG): the last arriver of a group (its ticket value
//     says so) sums the members' rows in member order and publishes the group row;
//   * the last arriving group combiner sums the NG group rows in group order -> AB = [WᵀX | WᵀW]
//     (deterministic: no order depends on arrival) and raises the iteration flag;
//   * every workgroup polls that flag (one lane, sc1 loads, s_sleep, bounded by a timeout that sets
//     an error word instead of hanging), reads AB (sc1) and applies the basis update itself, in
//     fp64 in LDS (SK:634-728; bit-identical arithmetic to basis_update_block), so H never makes
//     another round trip.
// Hand-off protocol: MI355X_MICROARCH.md "valid forms" table row 1 (sc1 stores, every storing wave
// `s_waitcnt vmcnt(0)`, a barrier, ONE lane's agent-scope add / flag store; sc1 loads by the
// consumer after its poll matched, the other waves behind a barrier).
// While the tail of the reduction runs, the first two tiles of the next iteration are already in
// LDS / in flight, so HBM keeps streaming across the iteration boundary.
// Residency: grid <= the occupancy query's co-resident capacity; every spin is bounded (error word).
// Counters (caller-owned, zero at rest): the last combiner of the launch zeroes them again.
// ------------------------------------------------------------------------------------------------
namespace sl {
constexpr int L_RED = L_TOTAL;                          // flush scratch [NWAVE*4][NR] fp32
constexpr int L_H = L_RED + (RED + 15) / 16 * 16;       // H fp64 [K][F]
constexpr int L_AB = L_H + K * F * 8;                   // AB fp64 [K][V]
constexpr int L_FLAG = L_AB + K * V * 8;                // 4 ints
constexpr int L_PTOTAL = L_FLAG + 16;
constexpr int GROUP = 16;                               // workgroups per first-level group
constexpr int MAX_GROUPS = 64;
constexpr uint32_t XPOISON = 0xFFFFFFFFu;                // exchange flag of a failed rank
constexpr uint64_t SPIN_TIMEOUT = 200000000ull;         // 2 s of s_memrealtime (100 MHz)
}  // namespace sl

// counter words (uint32): [0] reduce_kernel's ticket; the persistent kernel's at 128-byte strides
static_assert(sl::MAX_GROUPS <= NSLICE, "group rows live in the reduction stage buffer");
constexpr int CNT_GROUP0 = 32;
constexpr int CNT_TOP = CNT_GROUP0 + 32 * sl::MAX_GROUPS;
constexpr int CNT_FLAG = CNT_TOP + 32;
constexpr int CNT_ERR = CNT_FLAG + 32;
constexpr int DYN_GRP = 8;                       // workgroups per floating-tile pool
constexpr int DYN_MAX_POOLS = sl::GROUP * sl::MAX_GROUPS / DYN_GRP;
constexpr int CNT_POOL = CNT_ERR + 32;           // floating-tile pools [parity][pool] (32-word stride)
constexpr int CNT_RCOL0 = CNT_POOL + 2 * DYN_MAX_POOLS * 32;          // reduce_kernel: one ticket per 64-column block
constexpr int CNT_UPD = CNT_POOL;  // basis_update_split_kernel's ticket (the pools serve layout 3 only)
// the wave-tile kernels' XCC table (round 6): word b = 1 + the XCC id workgroup b runs on (written at
// the launch's start, zeroed by the launch's last combiner), in the pools' words past CNT_UPD's line
constexpr int CNT_XCC0 = CNT_POOL + 32;
constexpr int RED_MAX_COLS = 512;
constexpr int CNT_WORDS = CNT_RCOL0 + RED_MAX_COLS;
static_assert(CNT_XCC0 + sl::GROUP * sl::MAX_GROUPS <= CNT_RCOL0, "the XCC table fits the pools' words");

// sHt (fp32 [84][4], rows >= 81 zero) and sHHt (fp64 [4][4]) from the fp64 H in LDS; the HHᵀ
// arithmetic (lanes over f, fixed shuffle tree) is that of basis_update_block.
__device__ __forceinline__ void sl_derive_basis(unsigned char* smem, int t) {
  using namespace sl;
  const double* sH = reinterpret_cast<const double*>(smem + L_H);
  float* sHt = reinterpret_cast<float*>(smem + L_HT);
  double* sHHt = reinterpret_cast<double*>(smem + L_HHT);
  for (int e = t; e < NWAVE * NF * K; e += NT) {
    const int f = e / K;
    const int j = e - f * K;
    sHt[e] = f < F ? (float)sH[j * F + f] : 0.f;
  }
  const int lane = t & 63;
  const int wave = t >> 6;
  for (int e = wave; e < K * K; e += NWAVE) {
    const int j = e / K;
    const int m = e - j * K;
    double v = 0.0;
    for (int f = lane; f < F; f += 64) v = fma(sH[j * F + f], sH[m * F + f], v);
    v = wave_sum(v);
    if (lane == 0) sHHt[e] = v;
  }
  __syncthreads();
}

// H <- H·(WᵀX / ((WᵀW)·H (+l1)(+l2·H))) on the fp64 H in LDS from AB in LDS (SK:634-728)
__device__ __forceinline__ void sl_update_basis(unsigned char* smem, int t, double l1, double l2) {
  using namespace sl;
  double* sH = reinterpret_cast<double*>(smem + L_H);
  const double* sAB = reinterpret_cast<const double*>(smem + L_AB);
  double hn[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = t + NT * u;
    hn[u] = 0.0;
    if (e < K * F) {
      const int j = e / F;
      const int f = e - j * F;
      double h = sH[e];
      const double num = sAB[j * V + f];                                 // (WᵀX)[j][f], SK:639
      double den = 0.0;                                                  // ((WᵀW)·H)[j][f], SK:640
      for (int m = 0; m < K; ++m) den = fma(sAB[j * V + F + m], sH[m * F + f], den);
      if (l1 > 0.0) den += l1;                                           // SK:702-703
      if (l2 > 0.0) den = den + l2 * h;                                  // SK:704-705
      if (den == 0.0) den = EPS32;                                       // SK:706
      hn[u] = h * (num / den);                                           // SK:722-726
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (t + NT * u < K * F) sH[t + NT * u] = hn[u];
  __syncthreads();
  sl_derive_basis(smem, t);
}

struct PersistArgs {
  const float* X;
  float* W;
  double* H64;       // in: the basis; out: the final basis
  double* Ht;        // out [F][4]
  double* HHt;       // out [4][4]
  double* partials;  // [G][K*V] per-workgroup rows
  double* groups;    // [NG][K*V] group rows
  double* AB;        // [K*V]: in (apply_first) / out (the last iteration's reduced accumulators)
  uint32_t* cnt;     // CNT_WORDS counters
  int64_t n_tiles;
  int n_iter;
  int n_groups;
  int n_static;      // DYN: tiles per workgroup with W resident; tiles n_static*G.. float (the pool)
  double l1W, l2W, l1H, l2H;
  int apply_first;   // first apply the pending basis update from AB (multi-GPU: AB all-reduced)
  int apply_last;    // apply the last iteration's basis update in-launch (single GPU)
  // MULTI (one persistent launch per rank, the all-reduce in-launch): the exchange control block
  // (XC_* words, device memory), read only inside the exchange so that its values do not occupy
  // SGPRs through the streaming loop
  uint64_t* xctl;
  // TOL (the tolerance test on the device, SK:872-884): the control block of TC_* doubles
  double* tolctl;
  // the wave-tile kernel's first reduction level through the XCD's L2 (round 6):
  // a group's members (b ≡ g mod NG: one XCD under round-robin placement) store their partial rows
  // with plain stores, kept in the L2 their combiner reads with sc1 loads — from the second iteration
  // on, and only when the XCC table shows every member of the group on the combiner's XCC (placement
  // is never assumed: a group spread over XCDs keeps the write-through stores)
  int l2rows = 0;
};

// tolerance control block (doubles; TC_WSNAP holds a pointer's bits): inputs tol, it0 (global index
// of the launch's first iteration), the capacity of the error list; in/out the error at init and the
// previous checked error; outputs the iterations done, whether the test stopped the fit, whether
// the stopped fit's W is in the snapshot buffer (streamed W) rather than in W itself, the count and
// list of the checked errors (index g / 10 for the state after g iterations)
constexpr int TC_TOL = 0, TC_IT0 = 1, TC_INIT = 2, TC_PREV = 3, TC_DONE = 4, TC_STOPPED = 5, TC_IN_SNAP = 6,
              TC_WSNAP = 7, TC_CAP = 8, TC_NERR = 9, TC_ERRS = 16;
static_assert(TC_TOL == CNMF_TC_TOL && TC_IT0 == CNMF_TC_IT0 && TC_INIT == CNMF_TC_INIT && TC_PREV == CNMF_TC_PREV &&
                  TC_DONE == CNMF_TC_DONE && TC_STOPPED == CNMF_TC_STOPPED && TC_IN_SNAP == CNMF_TC_IN_SNAP &&
                  TC_WSNAP == CNMF_TC_WSNAP && TC_CAP == CNMF_TC_CAP && TC_NERR == CNMF_TC_NERR && TC_ERRS == CNMF_TC_ERRS,
              "tolerance control block slots = include/cnmf_hip.h");
constexpr uint32_t FLAG_STOP = 1u << 30;  // the iteration flag of a launch the tolerance test stopped

// exchange control block words: rank, world, byte offset of the flags in an exchange buffer, the
// generation base (advanced by n_iter at the end of every launch, on the device), then the
// world exchange-buffer pointers (this rank's own at XC_PEERS + rank)
constexpr int XC_RANK = 0, XC_WORLD = 1, XC_FLAG_OFF = 2, XC_GEN = 3, XC_PEERS = 8;

__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// two doubles as one 16-byte sc1 store (p 16-byte aligned; the MI355X guide's table: a 16-B sc1
// store costs about a plain one, 8-B accesses 0.54-0.70x the rate)
__device__ __forceinline__ void st16_sc1(double* p, double v0, double v1) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  const d2v v = d2v{v0, v1};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

// n / d for the W-updates of the wave-tile kernels: v_rcp_f64 + one Newton step (relative error
// ~2^-50, far below the fp32 rounding of the new w that follows) in place of the fp64 division's
// ~10-instruction IEEE sequence (round 5; d is a denominator >= EPS32, never denormal)
__device__ __forceinline__ double div_nr(double n, double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return n * r;
}

// The arguments of the bf16 wave-tile pass and of its persistent form (mu_iter_bfw_kernel).
struct BfwArgs {
  const bf16_t* X;
  float* W;
  const double* Ht;   // the pass: the basis (Hᵀ fp64 [F][16], HHᵀ [16][16])
  const double* HHt;
  double* partials;   // [G][k(F+k)]
  int64_t n_rows;
  int F, k;
  double l1, l2;
  int flags;
  int64_t n_tiles;    // full 64-sample tiles
  // PERSIST (mu_iter_bfw_kernel): n_iter MU iterations in ONE launch
  double* H64;        // in: the basis [k][F]; out: the final basis
  double* Ht_out;     // out: Hᵀ [F][16], HHᵀ [16][16] of the final basis
  double* HHt_out;
  double* AB;         // out: the last iteration's [WᵀX | WᵀW] (k(F+k))
  uint32_t* cnt;      // counters (at rest on entry, left at rest): CNT_GROUP0 / CNT_TOP = the two
                      // grid barriers of an iteration, CNT_ERR
  int n_iter;
  double l1H, l2H;
};

// KSC > 0: K-steps (and 2·KSC feature blocks) and KC components at compile time (cfg4: KSC = 10,
// F in 289..320, KC = 16): fully unrolled, branch-free phases the scheduler can interleave (with
// runtime bounds every K-step and feature block was its own basic block: phases 1 and 3 ran as
// dependent chains, 2647 and 2263 cycles per wave tile, profiles/r03/bfw/); KSC = 0: runtime F, k.
// PERSIST (KSC = 10, KC = 16 only): the n_iter iterations of mu_iter_bfw_kernel (below).
// NHT: H in NHT bf16 terms in phase 1.  Round 6 measured two terms (sixteen
// significant bits of H: a third fewer phase-1 MFMAs and H reads) and kept three: cfg4 1.7-4 %
// faster per iteration, but the dropped term's bias (the same rounding of H for every sample) moved
// W 5x further from the fp64 oracle — 2.3e-6 against 4.7e-7 after 40 iterations, 5.1e-6 against
// 1.9e-6 after cfg4's 500 (profiles/r06/cfg4_hterms/) — half the 1e-5 bar for 2-4 % of speed.
// CNMF_BFW_HTERMS=2 selects it in the diagnostic build.
template <int KSC, int KC, bool PERSIST, int NHT = 3>
__device__ __forceinline__ void bfw_run(const BfwArgs& a) {
  static_assert(NHT == 2 || NHT == 3, "H in two or three bf16 terms in phase 1");
  using namespace bw;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const bf16_t* __restrict__ X = a.X;
  float* __restrict__ W = a.W;
  double* __restrict__ partials = a.partials;
  int F = a.F, k = a.k;
  const double l1 = a.l1, l2 = a.l2;
  const int flags = PERSIST ? (CNMF_PASS_UPDATE_W | CNMF_PASS_ACCUMULATE) : a.flags;
  const int64_t n_tiles = a.n_tiles;
  const Lds L = lds(F);
  const int t = threadIdx.x;
  const int l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = l >> 4, li = l & 15;
  const int KS = KSC ? KSC : bm::ksteps(F);
  const int NB = KSC ? 2 * KSC : (F + 15) / 16;  // KSC: the last blocks past F read finite pads / rows
  if (KC) k = KC;
  const int nchx = 2 * F, nchw = 4 * k;  // 16-byte chunks of a wave tile's X and W
  const bool do_acc = (flags & CNMF_PASS_ACCUMULATE) != 0;
  // this wave's two slots (a pair of wave tiles per body): X tile [16][F] bf16 (+ zero pad), W [16][k]
  unsigned char* xsp[2] = {smem + L.slot + (2 * w) * L.slotb, smem + L.slot + (2 * w + 1) * L.slotb};
  const int XR = L.xrow;
  const unsigned xpad = (unsigned)(XR - 2 * F), mrow = (unsigned)((0x100000000ull + 2 * F - 1) / (2 * F));

  // ---- basis constants: H in three bf16 terms [n][32·KS] (zero beyond F / k), HHᵀ (as bm)
  double* sHHt = reinterpret_cast<double*>(smem + L.hht);
  double* sH64 = reinterpret_cast<double*>(smem + L.total);  // PERSIST: the fp64 basis [k][F]
  auto put_one = [&](int n, int f, double h) {
    const uint16_t h1 = bm::bf16_rn((float)h);
    const double r1 = h - (double)bm::bf16_f(h1);
    const uint16_t h2 = bm::bf16_rn((float)r1);
    const double r2 = r1 - (double)bm::bf16_f(h2);
    const uint16_t h3 = bm::bf16_rn((float)r2);
    uint16_t* row = reinterpret_cast<uint16_t*>(smem + L.hs + n * L.hrow) + f;
    row[0] = h1;
    row[bm::KP * L.hrow / 2] = h2;
    row[2 * bm::KP * L.hrow / 2] = h3;
  };
  auto put_terms = [&](auto hval) {
    for (int e = t; e < bm::KP * 32 * KS; e += NT) {
      const int n = e / (32 * KS);
      const int f = e - n * 32 * KS;
      put_one(n, f, (n < k && f < F) ? hval(n, f) : 0.0);
    }
  };
  // PERSIST: the terms and HHᵀ from the fp64 basis in LDS (thread = entry (j, m) of HHᵀ: four
  // interleaved chains over f combined in a fixed order — every workgroup the same bits, and HHᵀ
  // exactly symmetric)
  auto derive = [&]() {
    put_terms([&](int n, int f) { return sH64[n * F + f]; });
    const int j = t >> 4, m = t & 15;
    double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
    if (j < k && m < k) {
      const double* hj = sH64 + j * F;
      const double* hm = sH64 + m * F;
      int f = 0;
      for (; f + 4 <= F; f += 4) {
        c0 = fma(hj[f], hm[f], c0);
        c1 = fma(hj[f + 1], hm[f + 1], c1);
        c2 = fma(hj[f + 2], hm[f + 2], c2);
        c3 = fma(hj[f + 3], hm[f + 3], c3);
      }
      for (; f < F; ++f) c0 = fma(hj[f], hm[f], c0);
    }
    static_assert(NT == bm::KP * bm::KP, "one thread per HHᵀ entry");
    sHHt[t] = (c0 + c1) + (c2 + c3);
  };
  // the slots' zero pads: past the last row, and (never staged) each row's tail
  auto zero_pads = [&]() {
    if (l < 16) {
      reinterpret_cast<uint32_t*>(xsp[0] + TSW * XR)[l] = 0u;
      reinterpret_cast<uint32_t*>(xsp[1] + TSW * XR)[l] = 0u;
    }
    for (int e = l; e < TSW * (int)(xpad / 4); e += 64) {
      const int r = e / (int)(xpad / 4), c = e - r * (int)(xpad / 4);
      reinterpret_cast<uint32_t*>(xsp[0] + r * XR + 2 * F)[c] = 0u;
      reinterpret_cast<uint32_t*>(xsp[1] + r * XR + 2 * F)[c] = 0u;
    }
  };
  if constexpr (PERSIST) {
    for (int e = t; e < k * F; e += NT) sH64[e] = a.H64[e];
    __syncthreads();
    derive();
  } else {
    if constexpr (KSC != 0) {
      // the pass's head (round 6): all of this thread's Hᵀ loads in flight at once (clamped addresses,
      // no guard) — the loop above waited for each before issuing the next, one L2 round trip per
      // entry and 20 per thread at cfg4, in every per-iteration launch
      constexpr int NE = bm::KP * 32 * KSC, PER = (NE + NT - 1) / NT;
      double hv[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = t + NT * u;
        const int n = e / (32 * KSC), f = e - n * 32 * KSC;
        hv[u] = a.Ht[(size_t)min(f, F - 1) * bm::KP + min(n, bm::KP - 1)];
      }
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = t + NT * u;
        const int n = e / (32 * KSC), f = e - n * 32 * KSC;
        if (e < NE) put_one(n, f, (n < k && f < F) ? hv[u] : 0.0);
      }
    } else {
      put_terms([&](int n, int f) { return a.Ht[(size_t)f * bm::KP + n]; });
    }
    for (int e = t; e < bm::KP * bm::KP; e += NT) sHHt[e] = a.HHt[e];
  }
  zero_pads();
  __syncthreads();
  double hhb[4];  // B operand of the den MFMA: HHᵀ[m = 4kk + g][n = li]
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) hhb[kk] = sHHt[(4 * kk + g) * bm::KP + li];

  // ---- this wave's tiles: rows [64·(blockIdx + G·i) + 16w, +16), i < ntw (full 64-sample tiles)
  const int64_t G = gridDim.x;
  const int ntw = (int)((n_tiles - blockIdx.x + G - 1) / G);
  const unsigned char* Xb = reinterpret_cast<const unsigned char*>(X);
  const unsigned char* Wb = reinterpret_cast<const unsigned char*>(W);
  auto row0 = [&](int i) -> int64_t {  // first row of wave tile i (past the last: row 16w of tile 0)
    return 64 * (i < ntw ? (int64_t)blockIdx.x + G * i : (int64_t)blockIdx.x) + 16 * w;
  };
  auto prefetch = [&](u32x4 (&pf)[PFS], int i) {
    const int64_t r0 = row0(i);
    const unsigned char* xsrc = Xb + (size_t)r0 * F * 2;
#pragma unroll
    for (int u = 0; u < PFX; ++u) ld16(pf[u], xsrc + 16 * (l + 64 * u < nchx ? l + 64 * u : l));
    ld16(pf[PFX], Wb + (size_t)r0 * k * 4 + 16 * (l < nchw ? l : 0));
  };
  auto stage = [&](const u32x4 (&pf)[PFS], unsigned char* xs) {
    stage_x<0>((unsigned)(uintptr_t)xs, pf, l, nchx, mrow, xpad);
    // W [16][k]: at k = 16 the lane's chunk (s = l/4, j = l%4) goes to chunk j ^ ((s >> 1) & 3) of row s,
    // so phase 2's column reads (16 samples × 2 components per half-wave) spread over 16 banks, not 4
    const int wch = KC == 16 ? (l & ~3) | ((l & 3) ^ ((l >> 3) & 3)) : l;
    if (l < nchw) st16<0>((unsigned)(uintptr_t)(xs + L.xbytes + 16 * wch), pf[PFX]);
  };

  // accumulators: phase 3's fp32 MFMA chains over the wave's tiles (in AGPRs: no VALU touches
  // them before the end of the launch, so the 20 block chains run interleaved)
  f32x4 cacc[NBX], bacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int nb = 0; nb < NBX; ++nb) cacc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // invalid lanes' stores land in this workgroup's partial row (rewritten at the end of the launch;
  // the host guarantees k(F+k) >= 1024 doubles): every wave tile issues exactly NSTB stores per lane
  float* dummy = reinterpret_cast<float*>(partials + (size_t)blockIdx.x * k * (F + k)) + 64 * w + l;
  STAMP_DECL
  EOI_DECL

  // phase 1 for a PAIR of wave tiles: each K-step's three H terms are read from LDS once for both
  // tiles' chains (two independent MFMA chains; half the H traffic of one tile per body).  K-steps
  // run in pairs on separate accumulators (four independent chains), whose fp32 sum is folded into
  // fp64 once per pair of K-steps (round 5: half the fp64 converts and adds of a fold per K-step;
  // a fold now covers 64 features, as the wave-tile kernels' 7-feature chains cover 7 x k)
  auto phase1 = [&](double (&n0)[4], double (&n1)[4]) {
    const unsigned char* xa0 = xsp[0] + li * XR + 16 * g;
    const unsigned char* xa1 = xsp[1] + li * XR + 16 * g;
    const unsigned char* hb = smem + L.hs + li * L.hrow + 16 * g;
    auto kstep = [&](int ks, f32x4& u, f32x4& v) {
      const s16x8 a = *reinterpret_cast<const s16x8*>(xa0 + 64 * ks);  // 16-B aligned rows: one b128
      const s16x8 c = *reinterpret_cast<const s16x8*>(xa1 + 64 * ks);
      const bf16x8 b1 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(hb + 64 * ks));
      const bf16x8 b2 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(hb + bm::KP * L.hrow + 64 * ks));
      const bf16x8 av = __builtin_bit_cast(bf16x8, a), cv = __builtin_bit_cast(bf16x8, c);
      if constexpr (NHT == 3) {
        const bf16x8 b3 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(hb + 2 * bm::KP * L.hrow + 64 * ks));
        u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b3, u, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cv, b3, v, 0, 0, 0);
      }
      u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b2, u, 0, 0, 0);
      v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cv, b2, v, 0, 0, 0);
      u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b1, u, 0, 0, 0);
      v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cv, b1, v, 0, 0, 0);
    };
#pragma unroll
    for (int ks = 0; ks < (KSC ? KSC : 10); ks += 2) {
      if (!KSC && ks >= KS) break;
      const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 u0 = z, v0 = z, u1 = z, v1 = z;
      kstep(ks, u0, v0);
      if (KSC ? ks + 1 < KSC : ks + 1 < KS) kstep(ks + 1, u1, v1);
      const f32x4 u = u0 + u1, v = v0 + v1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        n0[r] += (double)u[r];
        n1[r] += (double)v[r];
      }
    }
  };
  // phases 2 and 3 of one wave tile (slot p, first row r0; invalid: w' = 0 and dummy stores)
  auto update = [&](int p, int64_t r0, bool valid, const double (&num64)[4]) {
    const unsigned char* xs = xsp[p];
    const float* wso = reinterpret_cast<const float*>(xs + L.xbytes);
    auto wix = [&](int s, int m) { return KC == 16 ? 16 * s + (m ^ (((s >> 1) & 3) << 2)) : s * k + m; };
    // phase 2: den = w·HHᵀ (f64 MFMA; A row ρ = li carries sample 4(ρ&3) + (ρ>>2), so D[g + 4r] is
    // sample 4g + r), then w' = w·num/den (SK:553-629) for (s = 4g + r, n = li)
    f64x4 den = f64x4{0.0, 0.0, 0.0, 0.0};
    const int sa = 4 * (li & 3) + (li >> 2);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int m = 4 * kk + g;
      const double av = m < k ? (double)wso[wix(sa, m)] : 0.0;
      den = __builtin_amdgcn_mfma_f64_16x16x4f64(av, hhb[kk], den, 0, 0, 0);
    }
    float wr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = 4 * g + r;
      float wn = 0.f;
      if (li < k) {
        double d = den[r];
        const double wold = (double)wso[wix(s, li)];
        if (l1 > 0.0) d += l1;              // SK:616-617
        if (l2 > 0.0) d = d + l2 * wold;    // SK:618-619
        if (d == 0.0) d = EPS32;            // SK:620
        wn = (float)(wold * div_nr(num64[r], d));  // SK:622-629 (div_nr: VERDICT r4 item 3b)
      }
      wn = valid ? wn : 0.f;
      wr[r] = wn;
      float* dst = (valid && li < k) ? W + (size_t)(r0 + s) * k + li : dummy + 256 * (r + 4 * p);
      *dst = wn;
    }
    if (!do_acc) return;
    // phase 3: A[m = 4g + r][f = 16nb + li] and B[m][n] over the tile's 16 samples
    // w'[4g + j][li] in TWO bf16 terms (16 significant bits; round 5): the dropped
    // third term is an unbiased per-sample rounding of |w'|·2^-18 at most, which the sum over the
    // samples averages out (relative error ~2^-17/sqrt(n) of A = W'ᵀX: 1e-8 at 1e6 rows), where phase
    // 1's H terms stay three (a rounding of H is the same for every sample: a bias, not noise)
    s16x4 a1, a2;  // the A operand (row m = li, k = 4g + j)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint16_t h1 = bm::bf16_rn(wr[j]);
      const float r1 = wr[j] - bm::bf16_f(h1);
      a1[j] = (short)h1;
      a2[j] = (short)bm::bf16_rn(r1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) bacc = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[r], wr[r], bacc, 0, 0, 0);
    const int q = li >> 2, pp = li & 3;
    const unsigned char* xb0 = xs + (4 * g + q) * XR + 8 * pp;
#pragma unroll
    for (int nb = 0; nb < NBX; ++nb) {
      if (nb < (KSC ? 2 * KSC : NB)) {
        const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xb0 + 32 * nb));
        cacc[nb] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a2, b, cacc[nb], 0, 0, 0);
        cacc[nb] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a1, b, cacc[nb], 0, 0, 0);
      }
    }
  };

  u32x4 pf[PD][PFS];
  static_assert(PD == 2, "a pair of wave tiles per body");
  static_assert(!PERSIST || (KSC == 10 && KC == 16), "the persistent form serves the cfg4 shape");
  const int np2 = (ntw + 1) & ~1;  // this wave's tiles per iteration rounded up to whole pairs
  prefetch(pf[0], 0);
  prefetch(pf[1], 1);
#pragma unroll
  for (int d = 0; d < 2 * NSTB; ++d)  // as if a body had run: the first waits count exactly
    asm volatile("global_store_dword %0, %1, off" ::"v"(dummy + 256 * d), "v"(0) : "memory");
  // PERSIST: the end-of-iteration scratch — the waves' sums, then AB, at LDS offset 0 (the slots and
  // the H terms are rebuilt before the next body stages anything), the reduce-scatter's row-chunk
  // sums after AB, the control words after the fp64 basis
  int* sFlag = reinterpret_cast<int*>(smem + L.total + align16((size_t)k * F * 8));
  double* red2 = reinterpret_cast<double*>(smem + align16((size_t)k * (F + k) * 8));
  const int n_it = PERSIST ? a.n_iter : 1;
  for (int it = 0; it < n_it; ++it) {
    for (int i0 = 0; i0 < ntw; i0 += 2) {
      STAMP(0);
      // younger than set 0: set 1's loads and the previous body's 2·NSTB stores; than set 1: the stores
      wait_set<PFS + 2 * NSTB>(pf[0]);
      stage(pf[0], xsp[0]);
      wait_set<2 * NSTB>(pf[1]);
      stage(pf[1], xsp[1]);
      STAMP(1);  // 1: waits + staging
      // the next body's pair; PERSIST, after the iteration's last body: the next iteration's first
      // pair (the same tiles: their W' of this iteration was stored >= 2 bodies earlier and has
      // retired at this body's waits — the host keeps >= 6 tiles per workgroup)
      const int nx = (PERSIST && i0 + 2 >= np2) ? 0 : i0 + 2;
      prefetch(pf[0], nx);
      prefetch(pf[1], nx + 1);
      STAMP(2);  // 2: prefetch issue
      double n0[4] = {0.0, 0.0, 0.0, 0.0}, n1[4] = {0.0, 0.0, 0.0, 0.0};
      phase1(n0, n1);
      STAMP(3);  // 3: phase 1 (both tiles)
      update(0, row0(i0), true, n0);
      STAMP(4);  // 4: phases 2 + 3 of the first tile
      update(1, row0(i0 + 1), i0 + 1 < ntw, n1);
      STAMP(5);  // 5: phases 2 + 3 of the second tile
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup / the iteration
    if (!do_acc) {
      STAMP_FLUSH;
      return;
    }

    if (PERSIST) EOI(0);
    // ---- the workgroup's partial row [k][F + k]: the waves' sums in the order (w0 + w2) + (w1 + w3),
    // through LDS in two chunks of feature blocks (no per-lane array of sums: the next iteration's
    // prefetch stays in its AGPRs), [wave][block of the chunk][r][lane] doubles from offset 0
    __syncthreads();  // every wave done with its slot: LDS is reused from offset 0
    double* red = reinterpret_cast<double*>(smem);
    const int V = F + k;
    double* prow = partials + (size_t)blockIdx.x * k * V;
    constexpr int NBT = NBX + 1, CH = (NBT + 1) / 2;  // 21 blocks (the last: B = W'ᵀW'), 11 per chunk
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        const int nb = ch * CH + q;
        if (nb < NBT)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            red[((w * CH + q) * 4 + r) * 64 + l] = (double)(nb < NBX ? cacc[nb < NBX ? nb : 0][r] : bacc[r]);
      }
      __syncthreads();
      // two adjacent lanes' values per thread (the same row m, features f and f + 1): one 16-byte
      // store when both are in the row and the pair is 16-byte aligned, else one 8-byte store each
      for (int o = 2 * t; o < CH * 4 * 64; o += 2 * NT) {
        const int q = o >> 8, r = (o >> 6) & 3, ln = o & 63;
        const int nb = ch * CH + q;
        if (nb >= NBT) continue;
        const int i0 = (q * 4 + r) * 64 + ln, WS = CH * 4 * 64;
        double v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h)
          v[h] = (red[i0 + h] + red[2 * WS + i0 + h]) + (red[WS + i0 + h] + red[3 * WS + i0 + h]);
        const int m = 4 * (ln >> 4) + r, lli = ln & 15;  // lli even
        int64_t at = -1, lim = 0;  // element offset of lane ln's value in the row, valid count
        if (nb < NBX) {
          const int f = 16 * nb + lli;
          if (m < k && f < F) at = (int64_t)m * V + f, lim = min(2, F - f);
        } else if (m < k && lli < k) {
          at = (int64_t)m * V + F + lli, lim = min(2, k - lli);
        }
        if (at < 0) continue;
        if (PERSIST) {  // read by other workgroups (any XCD) after barrier A: sc1 stores
          if (lim == 2 && (at & 1) == 0)
            st16_sc1(prow + at, v[0], v[1]);
          else
            for (int h = 0; h < lim; ++h) st_sc1(prow + at + h, v[h]);
        } else {
          for (int h = 0; h < lim; ++h) prow[at + h] = v[h];
        }
      }
      __syncthreads();
    }
    if constexpr (!PERSIST) {
      STAMP_FLUSH;
      return;
    } else {
      // ---- the end of an iteration (PERSIST).  (1) barrier A: every workgroup's partial row stored
      // (CNT_GROUP0 reaches (it + 1)·G); (2) reduce-scatter: workgroup b sums AB's columns
      // [b·CW, b·CW + CW) over the G rows in row order (row chunks, then the chunks in order) and
      // stores them; barrier B (CNT_TOP); (3) every workgroup loads AB and applies the basis update
      // (SK:634-728, fp64) to its copy of the basis in LDS — the same bits everywhere.  The last
      // iteration: only the workgroup whose barrier-B add came last applies the update, writes
      // H64 / Hᵀ / HHᵀ and zeroes the counters; the others leave.  Every wait is bounded (2 s)
      // and sets the error word (MI355X_MICROARCH.md valid forms row 1: sc1 stores, every storing
      // wave's vmcnt(0), a barrier, one lane's agent-scope add; sc1 polls and sc1 loads).
      const int NOUT = k * V;
      const int Gi = (int)G, b = (int)blockIdx.x;
      uint32_t* cA = a.cnt + CNT_GROUP0;
      uint32_t* cB = a.cnt + CNT_TOP;
      uint32_t* err = a.cnt + CNT_ERR;
      auto grid_wait = [&](uint32_t* c, uint32_t target, int slot) -> bool {
        if (t == 0) {
          int ok = 1;
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          while (true) {  // the counter and the error word in one batch: one round trip per round
            const uint32_t ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
            if (ev != 0u) {
              ok = 0;
              break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > sl::SPIN_TIMEOUT) {
              __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              ok = 0;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          sFlag[slot] = ok;
        }
        __syncthreads();
        return sFlag[slot] != 0;
      };
      EOI(1);  // 1: the waves' sums -> the partial row, stores issued
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      EOI(8);  // 8: the row's stores retired
      if (t == 0) __hip_atomic_fetch_add(cA, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!grid_wait(cA, (uint32_t)((it + 1) * Gi), 0)) return;
      EOI(2);  // 2: barrier A
      // (2) this workgroup's columns of AB
      const int CW = (NOUT + Gi - 1) / Gi;
      const int c0 = b * CW;
      const int ncols = max(0, min(CW, NOUT - c0));
      if (CW <= NT) {
        const int nrc = NT / CW;                // row chunks
        const int RPC = (Gi + nrc - 1) / nrc;   // rows per chunk
        const int c = t % CW, r = t / CW;
        double v = 0.0;
        if (r < nrc && c < ncols) {
          // the chunk's rows in batches of 11 loads in flight (the compiler does not re-order sc1
          // loads: every batch pays the cross-XCD latency once)
          const int r0 = r * RPC, r1 = min(Gi, r0 + RPC);
          for (int m = r0; m < r1; m += 11) {
            double x[11];
#pragma unroll
            for (int u = 0; u < 11; ++u) x[u] = ld_sc1(partials + (size_t)min(m + u, r1 - 1) * NOUT + c0 + c);
#pragma unroll
            for (int u = 0; u < 11; ++u) v += m + u < r1 ? x[u] : 0.0;
          }
        }
        if (r < nrc) red2[r * CW + c] = v;
        __syncthreads();
        if (t < ncols) {
          double sum = 0.0;
          for (int q = 0; q < nrc; ++q) sum += red2[q * CW + t];
          st_sc1(a.AB + c0 + t, sum);
        }
      } else {
        for (int c = t; c < ncols; c += NT) {
          double v = 0.0;
          for (int m = 0; m < Gi; m += 8) {
            double x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = ld_sc1(partials + (size_t)min(m + u, Gi - 1) * NOUT + c0 + c);
#pragma unroll
            for (int u = 0; u < 8; ++u) v += m + u < Gi ? x[u] : 0.0;
          }
          st_sc1(a.AB + c0 + c, v);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      EOI(3);  // 3: reduce-scatter
      const bool last_it = it + 1 == a.n_iter;
      if (t == 0) {
        const uint32_t old = __hip_atomic_fetch_add(cB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sFlag[2] = old == (uint32_t)(a.n_iter * Gi - 1);
      }
      __syncthreads();
      if (last_it) {
        if (!sFlag[2]) return;  // another workgroup finishes the launch
      } else if (!grid_wait(cB, (uint32_t)((it + 1) * Gi), 1)) {
        return;
      }
      EOI(4);  // 4: barrier B
      // (3) the basis update from AB (SK:634-728), basis_update_split_kernel's arithmetic on the f64
      // matrix cores: wave w takes H's 16-feature blocks nb ≡ w (mod 4) — per block den = (WᵀW)·H
      // (4 MFMAs, old H), the new block in place, and the block's HHᵀ partial (4 MFMAs) chained over
      // the wave's blocks in block order; the four waves' partials are summed in a fixed order
      double* sAB = reinterpret_cast<double*>(smem);
      for (int o0 = 0; o0 < NOUT; o0 += 11 * NT) {  // AB in batches of 11 loads per thread in flight
        double x[11];
#pragma unroll
        for (int u = 0; u < 11; ++u) x[u] = ld_sc1(a.AB + min(o0 + t + NT * u, NOUT - 1));
#pragma unroll
        for (int u = 0; u < 11; ++u)
          if (o0 + t + NT * u < NOUT) sAB[o0 + t + NT * u] = x[u];
      }
      __syncthreads();
      EOI(5);  // 5: AB -> LDS
      typedef double f64x4v __attribute__((ext_vector_type(4)));
      double* sblk = red2 + NT + w * (16 * 17);          // this wave's new block [j][f] (stride 17)
      double* hpart = red2 + NT + 4 * (16 * 17);         // [wave][16][16] HHᵀ partials
      {
        double bfr[4];  // A operand: (WᵀW)[j = li][m = 4kk + g]
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int m = 4 * kk + g;
          bfr[kk] = (li < k && m < k) ? sAB[li * V + F + m] : 0.0;
        }
        f64x4v hh = f64x4v{0.0, 0.0, 0.0, 0.0};
        const int NBF = (F + 15) / 16;
        for (int nb = w; nb < NBF; nb += 4) {
          const int f = 16 * nb + li;
          const bool fok = f < F;
          double hb[4], num[4], hold[4];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int m = 4 * kk + g;
            hb[kk] = (m < k && fok) ? sH64[m * F + f] : 0.0;  // H[m][f] (old)
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = g + 4 * r;
            const bool ok = j < k && fok;
            num[r] = ok ? sAB[j * V + f] : 0.0;  // (WᵀX)[j][f], SK:639
            hold[r] = ok ? sH64[j * F + f] : 0.0;
          }
          f64x4v den = f64x4v{0.0, 0.0, 0.0, 0.0};  // ((WᵀW)·H)[j][f], SK:640
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) den = __builtin_amdgcn_mfma_f64_16x16x4f64(bfr[kk], hb[kk], den, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int j = g + 4 * r;
            double h = hold[r];
            if (j < k && fok) {
              double d = den[r];
              if (a.l1H > 0.0) d += a.l1H;          // SK:702-703
              if (a.l2H > 0.0) d = d + a.l2H * h;   // SK:704-705
              if (d == 0.0) d = EPS32;              // SK:706
              h = h * (num[r] / d);                 // SK:722-726
              sH64[j * F + f] = h;
            }
            sblk[j * 17 + li] = (j < k && fok) ? h : 0.0;
          }
          // this block's HHᵀ: A[j = li][f = 4kk + g] = B[f][m = li] = h[li][4kk + g] (the wave's own
          // LDS writes above precede these reads)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const double v = sblk[li * 17 + 4 * kk + g];
            hh = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, hh, 0, 0, 0);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) hpart[(w * 16 + g + 4 * r) * 16 + li] = hh[r];  // P[j = g + 4r][m = li]
      }
      __syncthreads();
      sHHt[t] = (hpart[t] + hpart[256 + t]) + (hpart[512 + t] + hpart[768 + t]);
      __syncthreads();
      EOI(6);  // 6: the update
      if (last_it) {  // the basis state for the host, the counters back at rest
        const int KF = k * F;
        for (int e = t; e < KF; e += NT) a.H64[e] = sH64[e];
        for (int e = t; e < F * bm::KP; e += NT) {
          const int f = e / bm::KP, n = e - f * bm::KP;
          a.Ht_out[e] = n < k ? sH64[n * F + f] : 0.0;
        }
        a.HHt_out[t] = sHHt[t];
        if (t == 0) {
          __hip_atomic_store(cA, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(cB, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
      }
      put_terms([&](int n, int f) { return sH64[n * F + f]; });
      zero_pads();
      __syncthreads();
      EOI(7);  // 7: H terms, pads
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) hhb[kk] = sHHt[(4 * kk + g) * bm::KP + li];
#pragma unroll
      for (int nb = 0; nb < NBX; ++nb) cacc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      bacc = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

template <int KSC, int KC, int NHT = 3>
__global__ __launch_bounds__(NT, 1) void mu_pass_bfw_kernel(const bf16_t* __restrict__ X, float* __restrict__ W,
                                                            const double* __restrict__ Ht,
                                                            const double* __restrict__ HHt,
                                                            double* __restrict__ partials, int64_t n_rows, int F,
                                                            int k, double l1, double l2, int flags,
                                                            int64_t n_tiles) {
  BfwArgs a{};
  a.X = X;
  a.W = W;
  a.Ht = Ht;
  a.HHt = HHt;
  a.partials = partials;
  a.n_rows = n_rows;
  a.F = F;
  a.k = k;
  a.l1 = l1;
  a.l2 = l2;
  a.flags = flags;
  a.n_tiles = n_tiles;
  bfw_run<KSC, KC, false, NHT>(a);
}

// ------------------------------------------------------------------------------------------------
// mu_iter_bfw_kernel — cfg4 (bf16 X, F = 289..320, k = 16) as ONE persistent launch of n MU
// iterations: the wave-tile pass above with the cross-workgroup reduction and
// the basis update inside the launch, so an iteration has no kernel boundary, no separate
// reduction / update launch and no launch gap.  The next iteration's first pair of tiles is already
// in flight (AGPRs) while the workgroups meet; every workgroup keeps its own fp64 copy of the basis
// in LDS.  One workgroup per CU (the grid co-resident: the host checks the occupancy query).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NT, 1) void mu_iter_bfw_kernel(BfwArgs a) { bfw_run<10, 16, true>(a); }

// out[o] = Σ_m rows[m][o] in m order for the rows m = m0, m0 + step, ... (cnt rows); sc1 loads.
// Batches of 16 rows for both of a thread's outputs are issued before any is summed (row index
// clamped and the extra terms dropped after the load, so no load sits behind a branch).
__device__ __forceinline__ void sum_rows_sc1(const double* rows, int m0, int step, int cnt, double* lds_out,
                                             double* g_out, int t) {
  using namespace sl;
  constexpr int n_out = K * V;
  constexpr int RB = 16;
  static_assert(n_out <= 2 * NT, "two outputs per thread");
  const int o0 = t;
  const int o1 = t + NT < n_out ? t + NT : t;
  double v0 = 0.0, v1 = 0.0;
  for (int m = 0; m < cnt; m += RB) {
    double x0[RB], x1[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int r = m0 + min(m + u, cnt - 1) * step;
      x0[u] = ld_sc1(rows + (size_t)r * n_out + o0);
      x1[u] = ld_sc1(rows + (size_t)r * n_out + o1);
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      v0 += m + u < cnt ? x0[u] : 0.0;
      v1 += m + u < cnt ? x1[u] : 0.0;
    }
  }
  if (lds_out) lds_out[o0] = v0;
  st_sc1(g_out + o0, v0);
  if (t + NT < n_out) {
    if (lds_out) lds_out[o1] = v1;
    st_sc1(g_out + o1, v1);
  }
}

#ifdef CNMF_STAMPS
// diagnostic timeline of the persistent kernel (s_memrealtime, 100 MHz): per iteration and
// workgroup [0] = rows published (arrival), [1] = next iteration's basis ready (resume); per
// iteration the top combiner's AB publish time.  Never in the product build.
constexpr int TL_IT = 64, TL_WG = 2048;
__device__ unsigned long long g_tl[TL_IT * TL_WG * 2];
__device__ unsigned long long g_tl_pub[TL_IT];
__device__ unsigned long long g_tl_x[TL_IT * 4];  // MULTI exchange: start, stored, flags seen, summed
__device__ unsigned long long g_tl_start[TL_WG];
__device__ unsigned int g_tl_hw[TL_WG * 2];  // HW_REG_HW_ID (cu / sh / se bits), HW_REG_XCC_ID
#define TL(it_, slot_)                                                                          \
  do {                                                                                          \
    if (t == 0 && (it_) < TL_IT && b < TL_WG) g_tl[((it_) * TL_WG + b) * 2 + (slot_)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define TL_PUB(it_) do { if (t == 0 && (it_) < TL_IT) g_tl_pub[it_] = __builtin_amdgcn_s_memrealtime(); } while (0)
// per-level stamps of the reduction tree (round 6): [it][g][0] group g's combiner's ticket returned,
// [1] its group row stored (vmcnt(0) + barrier); [it][TL_LVG][0] the top's ticket returned, [1] AB summed
// and stored; and [it][wg] each workgroup's time before its partial-row stores (g_tl_pre)
constexpr int TL_LVG = 64;
__device__ unsigned long long g_tl_lv[TL_IT * (TL_LVG + 1) * 2];
__device__ unsigned long long g_tl_pre[TL_IT * TL_WG];
__device__ unsigned long long g_tl_seen[TL_IT * TL_WG];  // flag seen (non-top workgroups)
__device__ unsigned long long g_tl_ab[TL_IT * TL_WG];    // AB in LDS (non-top workgroups)
__device__ unsigned long long g_tl_upd[TL_IT * TL_WG];   // basis update done (before load_basis)
#define TL_LV(it_, g_, slot_)                                                                   \
  do {                                                                                          \
    if (t == 0 && (it_) < TL_IT) g_tl_lv[((it_) * (TL_LVG + 1) + (g_)) * 2 + (slot_)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define TL_PRE(it_) do { if (t == 0 && (it_) < TL_IT && b < TL_WG) g_tl_pre[(it_) * TL_WG + b] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define TL_SEEN(it_) do { if (t == 0 && (it_) < TL_IT && b < TL_WG) g_tl_seen[(it_) * TL_WG + b] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define TL_AB(it_) do { if (t == 0 && (it_) < TL_IT && b < TL_WG) g_tl_ab[(it_) * TL_WG + b] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define TL_UPD(it_) do { if (t == 0 && (it_) < TL_IT && b < TL_WG) g_tl_upd[(it_) * TL_WG + b] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define TL_X(it_, slot_) do { if (t == 0 && (it_) < TL_IT) g_tl_x[(it_) * 4 + (slot_)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define TL_START                                                                               \
  do {                                                                                         \
    if (t == 0 && b < TL_WG) {                                                                 \
      g_tl_start[b] = __builtin_amdgcn_s_memrealtime();                                        \
      unsigned hw_, xcc_;                                                                      \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                        \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                      \
      g_tl_hw[2 * b] = hw_;                                                                    \
      g_tl_hw[2 * b + 1] = xcc_;                                                               \
    }                                                                                          \
  } while (0)
#else
#define TL(it_, slot_) do {} while (0)
#define TL_PUB(it_) do {} while (0)
#define TL_X(it_, slot_) do {} while (0)
#define TL_START do {} while (0)
#define TL_LV(it_, g_, slot_) do {} while (0)
#define TL_PRE(it_) do {} while (0)
#define TL_SEEN(it_) do {} while (0)
#define TL_AB(it_) do {} while (0)
#define TL_UPD(it_) do {} while (0)
#endif

// The cross-rank all-reduce of AB (k(F+k) fp64) inside a persistent launch, run by the top
// combiner's NT threads after the rank's own AB is in sAB (LDS) and a.AB.  Each fp64 value travels
// as two 64-bit words {generation tag : 32-bit half}, written with system-scope atomic stores into
// slot `rank` of every rank's exchange buffer (remote stores over xGMI); a reader polls its own
// buffer until every word of every slot carries this generation's tag, so no separate flag, fence or
// store acknowledgement sits on the critical path.  Slots are summed in rank order: the same AB, bit
// for bit, on every rank.  Slots alternate by generation parity: rank p writes generation g+2 only
// after it has read every rank's g+1 words, which each rank writes only after it has read its
// generation-g slots.  A rank whose launch has failed tags its words XPOISON, which makes every peer
// fail too (no rank waits out its timeout per iteration).  The thread <-> element mapping is
// sum_rows_sc1's (o = t, t + NT).  Leaves the summed AB in sAB and a.AB.
__device__ __forceinline__ void xchg_allreduce_ab(uint64_t* xctl, double* AB, double* sAB, uint32_t* err, int it, int t) {
  using namespace sl;
  constexpr int n_out = K * V;
  static_assert(n_out <= 2 * NT && n_out > NT, "two elements per thread");
  // atomics: loaded here, not hoisted to the kernel entry
  const int xrank = (int)__hip_atomic_load(xctl + XC_RANK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int xworld = (int)__hip_atomic_load(xctl + XC_WORLD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t gen =
      (uint32_t)__hip_atomic_load(xctl + XC_GEN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (uint32_t)it + 1u;
  auto peer = [&](int r) {
    return reinterpret_cast<uint64_t*>(
        __hip_atomic_load(xctl + XC_PEERS + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  };
  TL_X(it, 0);
  const bool has1 = t + NT < n_out;
  const size_t slot = 2 * (size_t)n_out;  // words per rank slot
  const size_t par = (size_t)(gen & 1u) * xworld * slot;
  {
    const bool bad = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    const uint64_t tag = (uint64_t)(bad ? XPOISON : gen) << 32;
    const uint64_t b0 = (uint64_t)__double_as_longlong(sAB[t]);
    const uint64_t b1 = has1 ? (uint64_t)__double_as_longlong(sAB[t + NT]) : 0ull;
    for (int pr = 0; pr < xworld; ++pr) {
      uint64_t* dst = peer(pr) + par + (size_t)xrank * slot;
      __hip_atomic_store(dst + 2 * t, tag | (b0 & 0xFFFFFFFFull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(dst + 2 * t + 1, tag | (b0 >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (has1) {
        __hip_atomic_store(dst + 2 * (t + NT), tag | (b1 & 0xFFFFFFFFull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(dst + 2 * (t + NT) + 1, tag | (b1 >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  TL_X(it, 1);
  const uint64_t* mine = peer(xrank) + par;
  double v0 = 0.0, v1 = 0.0;
  constexpr int QB = 4;  // ranks polled per round (their loads in flight together)
  for (int q0 = 0; q0 < xworld; q0 += QB) {
    uint64_t w[QB][4];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
      const uint32_t ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // same batch
  #pragma unroll
      for (int j = 0; j < QB; ++j) {
        const uint64_t* src = mine + (size_t)min(q0 + j, xworld - 1) * slot;
        w[j][0] = __hip_atomic_load(src + 2 * t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w[j][1] = __hip_atomic_load(src + 2 * t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const int o1 = has1 ? t + NT : t;
        w[j][2] = __hip_atomic_load(src + 2 * o1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w[j][3] = __hip_atomic_load(src + 2 * o1 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      bool ok = true, poison = false;
  #pragma unroll
      for (int j = 0; j < QB; ++j)
  #pragma unroll
        for (int m = 0; m < 4; ++m) {
          const uint32_t tg = (uint32_t)(w[j][m] >> 32);
          ok = ok && tg == gen;
          poison = poison || tg == XPOISON;
        }
      if (ok) break;
      if (poison) {
        __hip_atomic_store(err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      if (ev != 0u) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TIMEOUT) {
        __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  #pragma unroll
    for (int j = 0; j < QB; ++j) {
      if (q0 + j < xworld) {  // rank order
        v0 += __longlong_as_double((long long)((w[j][1] << 32) | (w[j][0] & 0xFFFFFFFFull)));
        v1 += __longlong_as_double((long long)((w[j][3] << 32) | (w[j][2] & 0xFFFFFFFFull)));
      }
    }
  }
  TL_X(it, 2);
  sAB[t] = v0;
  st_sc1(AB + t, v0);
  if (has1) {
    sAB[t + NT] = v1;
    st_sc1(AB + t + NT, v1);
  }
  TL_X(it, 3);
}

// WRES: W stays resident in LDS for the whole launch (this workgroup's tiles, loaded once at the
// start and written back once at the end): the passes stream only X, 324 instead of 356 bytes per
// sample ("keep tensors resident instead of re-reading them").  Needs nbt·1 KB of extra LDS.
//
// TEAMS = 2: one 8-wave workgroup per CU made of two 4-wave teams, each running the tile pipeline
// below on its own tiles and its own copy of the LDS layout (team 1's at smem + team_lds), in
// lockstep: every barrier is the workgroup's.  Two independent 4-wave workgroups on a CU drift
// apart (one of the pair finishes several microseconds after the other, and the iteration waits
// for the slowest); in lockstep the pair shares the CU evenly.  The teams own virtual blocks
// vb = 2b + team (tiles vb + 2G·i); the team with one tile fewer runs a padding step (nothing
// stored, nothing accumulated) so both execute the same barriers.  The two teams' accumulators
// are combined into the workgroup's one fp64 row in a fixed order (deterministic).
#ifndef CNMF_TEAM_PRIO
#define CNMF_TEAM_PRIO 1
#endif
constexpr bool SETPRIO = CNMF_TEAM_PRIO != 0;
//
// DYN (floating tiles): each workgroup owns n_static tiles b + G·i (W resident, as above); the
// remaining tiles form a pool that the workgroups draw from one at a time, every iteration, with an
// agent-scope atomic counter (one per iteration parity).  A workgroup that streams faster takes more
// of them, so the iteration no longer waits for the slowest CU's fixed share (the per-CU / per-XCD
// spread of DESIGN.md §3.0).  A floating tile's W travels through HBM: sc1 loads and stores (the
// next iteration's owner may sit on another XCD; the hand-off rides the iteration's tickets and
// flag).  The draw for a position is issued one tile before it is needed (its latency hidden behind
// a tile), before that tile's prefetch loads (so waiting for it never waits for them); thread 0
// hands the result over through LDS.  The summation order then depends on the draw: results agree
// with the static layouts to fp32 summation-order noise but are not bit-repeatable.
template <int PD, bool WRES, bool MULTI = false, int TEAMS = 1, bool DYN = false>
__global__ __launch_bounds__(NT * TEAMS, TEAMS == 2 ? 1 : (PD == 1 ? 3 : 2)) void mu_iter_sl_kernel(PersistArgs a) {
  using namespace sl;
  static_assert(TEAMS == 1 || (TEAMS == 2 && PD == 2), "two teams: PD = 2");
  static_assert(!DYN || (TEAMS == 1 && PD == 2 && WRES), "floating tiles: pairs, PD = 2, W resident");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_base[];
  const int tid = threadIdx.x;
  const int team = TEAMS == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid >> 8);
  const int t = TEAMS == 1 ? tid : (tid & (NT - 1));
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int b = blockIdx.x;
  const int G = gridDim.x;
  const int NG = a.n_groups;
  const int g = b % NG;                          // group members: g, g + NG, g + 2 NG, ...
  const int gs = (G - g + NG - 1) / NG;
  const unsigned char* Xb = reinterpret_cast<const unsigned char*>(a.X);
  const unsigned char* Wb = reinterpret_cast<const unsigned char*>(a.W);
  // tiles of this team: vb + Gv·i, i < nbt_team; the loop runs nbt (team 0's count) steps per
  // iteration, the same every iteration.  The host guarantees nbt_team >= PD + 2, so a tile's W was
  // stored at least one tile before it is prefetched again.
  const int Gv = G * TEAMS;
  const int vb = b * TEAMS + team;
  const int nbt = (int)((a.n_tiles - (int64_t)b * TEAMS + Gv - 1) / Gv);
  const int nbt_team = TEAMS == 1 ? nbt : (int)((a.n_tiles - vb + Gv - 1) / Gv);
  const int nbt_max = (int)((a.n_tiles + Gv - 1) / Gv);
  const int team_lds = L_PTOTAL + (WRES ? nbt_max * WB : 0);  // the host sizes TEAMS x this
  unsigned char* smem = smem_base + (TEAMS == 1 ? 0 : team * team_lds);
  double* sH = reinterpret_cast<double*>(smem + L_H);
  double* sAB = reinterpret_cast<double*>(smem + L_AB);
  int* sFlag = reinterpret_cast<int*>(smem_base + L_FLAG);  // the workgroup's (team 0's copy)
  uint32_t* cnt_group = a.cnt + CNT_GROUP0 + 32 * g;
  uint32_t* cnt_top = a.cnt + CNT_TOP;
  uint32_t* flag = a.cnt + CNT_FLAG;
  uint32_t* err = a.cnt + CNT_ERR;
  // DYN pools: workgroups 8p..8p+7 (consecutive, so on different XCDs) share pool p, which holds
  // the floating tiles [f0, f1) (a share proportional to its workgroups); one counter per pool and
  // iteration parity, so ~n_float/64 draws land on each address instead of all on one (draws on one
  // address serialise at ~9 ns each: 4000 per iteration cost 37 µs)
  const int S = DYN ? a.n_static : 0;
  const int n_float = DYN ? (int)(a.n_tiles - (int64_t)S * G) : 0;
  const int n_pools = (G + DYN_GRP - 1) / DYN_GRP;
  const int my_pool = b / DYN_GRP;
  const int f0 = DYN ? S * G + (int)((int64_t)n_float * (my_pool * DYN_GRP) / G) : 0;
  const int f_n = DYN ? S * G + (int)((int64_t)n_float * min(my_pool * DYN_GRP + DYN_GRP, G) / G) - f0 : 0;
  uint32_t* pool = a.cnt + CNT_POOL + 32 * my_pool;  // + 32·DYN_MAX_POOLS for odd iterations
  const int n_res = DYN ? S : nbt_team;  // W tiles resident in LDS

  // ---- the basis for the first iteration
  for (int e = t; e < K * F; e += NT) sH[e] = a.H64[e];
  if (a.apply_first)
    for (int e = t; e < K * V; e += NT) sAB[e] = a.AB[e];
  if (t < 4) reinterpret_cast<float*>(smem + L_X + XB)[t] = 0.f;
  __syncthreads();
  if (a.apply_first)
    sl_update_basis(smem, t, a.l1H, a.l2H);
  else
    sl_derive_basis(smem, t);

  float acc[NC][K];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < K; ++j) acc[c][j] = 0.f;
  float acc33 = 0.f;

  const int total = a.n_iter * nbt;
  auto tile_at = [&](int q) -> int64_t {
    const int i = q % nbt;
    return vb + (int64_t)Gv * (TEAMS == 1 ? i : min(i, nbt_team - 1));  // padding step: a valid tile
  };
  unsigned char* wres = smem + L_PTOTAL;  // [nbt][64][4] fp32 when WRES
  if (WRES) {
    for (int c = t; c < n_res * (WB / 16); c += NT) {
      const int i = c / (WB / 16), ch = c - i * (WB / 16);
      *reinterpret_cast<u32x4*>(wres + i * WB + 16 * ch) =
          *reinterpret_cast<const u32x4*>(Wb + (size_t)(vb + (int64_t)Gv * i) * WB + 16 * ch);
    }
  }
  // DYN: the positions q, q+1, q+2 of this workgroup's tile sequence (tile, iteration, index in the
  // iteration; it == n_iter: past the end) and the generator of the next positions
  struct Pos {
    int tile, it, i;
  };
  int gen_it = 0, gen_i = 0;
  bool grab_pending = false;  // a draw was issued in the previous body (its value: thread 0's grab_reg)
  uint32_t grab_reg = 0;
  auto issue_grab = [&]() {
    if (tid == 0)
      grab_reg = __hip_atomic_fetch_add(pool + 32 * DYN_MAX_POOLS * (gen_it & 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    grab_pending = true;
  };
  auto produce = [&]() -> Pos {
    if (gen_it >= a.n_iter) return Pos{0, a.n_iter, 0};
    if (gen_i >= S) {  // a floating position: the draw issued one body ago (LDS word sFlag[3])
      const uint32_t got = (uint32_t)__builtin_amdgcn_readfirstlane(sFlag[3]);
      if (got < (uint32_t)f_n) {
        const Pos p{f0 + (int)got, gen_it, gen_i};
        ++gen_i;
        issue_grab();
        return p;
      }
      ++gen_it;  // the pool is empty: this workgroup's iteration ends here
      gen_i = 0;
      if (gen_it >= a.n_iter) return Pos{0, a.n_iter, 0};
    }
    const Pos p{b + G * gen_i, gen_it, gen_i};
    ++gen_i;
    if (gen_i == S) issue_grab();
    return p;
  };
  Pos P0{0, 0, 0}, P1{0, 0, 0}, P2{0, 0, 0};
  u32x4 pfA[PFN], pfB[PFN];
  uint64_t pwA[2] = {0, 0}, pwB[2] = {0, 0};  // DYN: the W chunk of the tile in pfA / pfB
  if (DYN) {
    P0 = produce();
    P1 = produce();
    P2 = produce();  // S >= PD + 2: all static
    sl_prefetch<false>(pfA, Xb, Wb, P0.tile, t);
    sl_prefetch<false>(pfB, Xb, Wb, P1.tile, t);
    sl_prefetch_w(pwB, Xb, Wb, P1.tile, false, t);
    sl_stage<false>(smem, 0, pfA, t);
    sl_prefetch<false>(pfA, Xb, Wb, P2.tile, t);
    sl_prefetch_w(pwA, Xb, Wb, P2.tile, false, t);
  } else {
    sl_prefetch<!WRES>(pfA, Xb, Wb, tile_at(0), t);
    if (PD == 2 && total > 1) sl_prefetch<!WRES>(pfB, Xb, Wb, tile_at(1), t);
    sl_stage<!WRES>(smem, 0, pfA, t);
    if (total > PD) sl_prefetch<!WRES>(pfA, Xb, Wb, tile_at(PD == 1 ? 1 : 2), t);
  }
  lds_barrier();
  TL_START;
  // the second-dispatched half (waves 4-7) loses every VALU arbitration to its older SIMD partner
  // at equal priority: one static raise, no per-segment flips (MI355X_MICROARCH.md, two waves per
  // SIMD, item 4)
  if (TEAMS == 2 && SETPRIO && team == 1) __builtin_amdgcn_s_setprio(1);

  bool alive = true;
  int wpar = 0;
  auto body = [&](int q, u32x4 (&pf)[PFN], uint64_t (&pw)[2]) {
    const int it = DYN ? P0.it : q / nbt;
    const int i = DYN ? P0.i : q - it * nbt;
    const bool end_it = DYN ? P1.it != P0.it : i + 1 == nbt;
    const bool last_it = it + 1 == a.n_iter;
    const bool has1 = DYN ? P1.it < a.n_iter : q + 1 < total;
    const bool hasP = DYN ? true : q + 1 + PD < total;
    const int64_t tile = DYN ? (int64_t)P0.tile : tile_at(q);
    const bool flt = DYN && i >= S;  // a floating tile: W staged from HBM, stored sc1
    const bool flt1 = DYN && P1.i >= S;
    float xv[NC];
    // two teams run half a tile apart: team 1 passes one barrier before its first tile of the
    // iteration and team 0 one after its last, so team 1's phase 1 overlaps team 0's phase 2 and
    // staging (and vice versa) instead of both teams hitting the same resources at once
    if (TEAMS == 2 && team == 1 && i == 0) lds_barrier();
    phase1(smem, xv, wave, lane);
    // this wave's W store of the previous tile has landed (vmcnt retires in order; at most the 6
    // loads issued after it may remain) before any wave passes barrier A and prefetches W again
    if (!WRES) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    lds_barrier();  // A
    phase2(smem, a.W, tile, wpar, wave, lane, a.l1W, a.l2W,
           // DYN: a floating tile's W is read from (and its update also written to) its staging slot
           DYN ? reinterpret_cast<float*>(flt ? smem + L_W + wpar * WB : wres + i * WB)
               : (WRES ? reinterpret_cast<float*>(wres + i * WB) : nullptr),
           TEAMS == 1 || i < nbt_team, flt);
    if (DYN) {
      if (has1) {
        sl_stage<false>(smem, wpar ^ 1, pf, t);
        sl_stage_w(smem, wpar ^ 1, pw, t);
      }
      // the draw issued in the previous body -> LDS, here where the stage has already waited for
      // the loads issued before it (a wait for the draw's value elsewhere in the body costs the
      // compiler's conservative vmcnt(0): the whole prefetch, ~0.8 µs per tile)
      if (grab_pending) {
        if (tid == 0) sFlag[3] = (int)grab_reg;
        grab_pending = false;
      }
    } else {
      if (has1) sl_stage<!WRES>(smem, wpar ^ 1, pf, t);
      if (hasP && !end_it) sl_prefetch<!WRES>(pf, Xb, Wb, tile_at(q + 1 + PD), t);
    }
    lds_barrier();  // B
    if (DYN) {  // position q + 1 + PD: its draw (if floating) read from LDS, the next draw issued
      const Pos P3 = produce();
      // at the iteration's end the prefetch waits until the row's vmcnt(0) below has passed
      if (!end_it && P3.it < a.n_iter) {
        sl_prefetch<false>(pf, Xb, Wb, P3.tile, t);
        sl_prefetch_w(pw, Xb, Wb, P3.tile, P3.i >= S, t);
      }
      P0 = P1;
      P1 = P2;
      P2 = P3;
    }
    phase3(smem, xv, acc, acc33, wave, lane);
    wpar ^= 1;
    if (!end_it) return;
    if (TEAMS == 2 && team == 0) lds_barrier();  // team 1's last tile

    // ---- end of the iteration: publish this workgroup's row, then the in-launch reduction
    flush_acc<true, TEAMS>(reinterpret_cast<float*>(smem + L_RED), acc, acc33, a.partials + (size_t)b * (K * V),
                           wave, lane, t, reinterpret_cast<const float*>(smem_base + L_RED),
                           reinterpret_cast<const float*>(smem_base + team_lds + L_RED), tid);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < K; ++j) acc[c][j] = 0.f;
    acc33 = 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores landed
    __syncthreads();
    // in flight during the reduction (DYN: P2 is now position q + 1 + PD)
    if (DYN) {
      if (P2.it < a.n_iter) {
        sl_prefetch<false>(pf, Xb, Wb, P2.tile, t);
        sl_prefetch_w(pw, Xb, Wb, P2.tile, P2.i >= S, t);
      }
    } else if (hasP) {
      sl_prefetch<!WRES>(pf, Xb, Wb, tile_at(q + 1 + PD), t);
    }
    TL(it, 0);
    if (tid == 0) {
      const uint32_t old = __hip_atomic_fetch_add(cnt_group, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sFlag[0] = old == (uint32_t)((it + 1) * gs - 1);
      sFlag[1] = 0;
      sFlag[2] = 1;
    }
    __syncthreads();
    if (sFlag[0]) {  // group combiner
      if (team == 0) sum_rows_sc1(a.partials, g, NG, gs, nullptr, a.groups + (size_t)g * (K * V), t);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const uint32_t old = __hip_atomic_fetch_add(cnt_top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sFlag[1] = old == (uint32_t)((it + 1) * NG - 1);
      }
      __syncthreads();
      if (sFlag[1] && team == 0) {  // top combiner: AB (team 0; team 1 copies it below)
        sum_rows_sc1(a.groups, 0, 1, NG, sAB, a.AB, t);
        if (MULTI) xchg_allreduce_ab(a.xctl, a.AB, sAB, err, it, t);
      }
      if (sFlag[1]) {
        // this iteration's pool is drained (every workgroup's failed draw precedes its ticket):
        // ready for iteration it + 2
        if (DYN && tid < n_pools)
          __hip_atomic_store(a.cnt + CNT_POOL + 32 * (DYN_MAX_POOLS * (it & 1) + tid), 0u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0 && !last_it)
          __hip_atomic_store(flag, (uint32_t)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        TL_PUB(it);
        if (TEAMS == 2) {  // team 1's copy of AB
          if (team == 1)
            for (int e = t; e < K * V; e += NT) sAB[e] = reinterpret_cast<const double*>(smem_base + L_AB)[e];
          __syncthreads();
        }
      }
    }
    const bool top = sFlag[1] != 0;
    if (last_it) {
      alive = false;
      if (WRES) {  // this team's W back to HBM, once per launch
        for (int c = t; c < n_res * (WB / 16); c += NT) {
          const int ii = c / (WB / 16), ch = c - ii * (WB / 16);
          *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned char*>(a.W) + (size_t)(vb + (int64_t)Gv * ii) * WB + 16 * ch) =
              *reinterpret_cast<const u32x4*>(wres + ii * WB + 16 * ch);
        }
      }
      if (!top) return;
      // the last combiner of the launch: every other workgroup has arrived for the last time
      if (a.apply_last) sl_update_basis(smem, t, a.l1H, a.l2H);
      if (team != 0) return;
      for (int e = t; e < K * F; e += NT) a.H64[e] = sH[e];
      for (int e = t; e < F * K; e += NT) {
        const int f = e / K;
        const int j = e - f * K;
        a.Ht[e] = sH[j * F + f];
      }
      if (t < K * K) a.HHt[t] = reinterpret_cast<const double*>(smem + L_HHT)[t];
      if (t < NG) __hip_atomic_store(a.cnt + CNT_GROUP0 + 32 * t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tid == 0) {
        __hip_atomic_store(cnt_top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (MULTI)  // the next launch's generations follow this one's
          __hip_atomic_fetch_add(a.xctl + XC_GEN, (uint64_t)a.n_iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (!top) {
      if (tid == 0) {
        const uint32_t want = (uint32_t)(it + 1);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (true) {  // the flag and the error word in one batch: one round trip per round
          const uint32_t ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) break;
          if (ev != 0u) {
            sFlag[2] = 0;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TIMEOUT) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sFlag[2] = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      if (!sFlag[2]) {  // a workgroup never arrived (not co-resident): give up, error word set
        alive = false;
        return;
      }
      for (int e = t; e < K * V; e += NT) sAB[e] = ld_sc1(a.AB + e);
      __syncthreads();
    }
    sl_update_basis(smem, t, a.l1H, a.l2H);
    TL(it, 1);
  };

  if (DYN) {
    for (int q = 0; alive; q += 2) {  // ends at the last iteration's end (or an error)
      body(q, pfB, pwB);
      if (alive) body(q + 1, pfA, pwA);
    }
  } else {
    for (int q = 0; q < total && alive; q += 2) {
      if (PD == 1) body(q, pfA, pwA);
      else body(q, pfB, pwB);
      if (q + 1 < total && alive) body(q + 1, pfA, pwA);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
}

// ------------------------------------------------------------------------------------------------
// mu_iter_wt_kernel<PD, MULTI> — the headline shape (fp32 X, F = 81, k = 4) as ONE persistent launch
// of barrier-free WAVE tiles.
//
// Why: the workgroup-tile kernel above (mu_iter_sl_kernel) is issue/latency-bound, not HBM-bound —
// with X served from L2 it runs at the same 67 µs per iteration (profiles/r02/probes/l2diag.log),
// its waves park 46 % of their cycles on two workgroup barriers per tile and on one-deep LDS reads
// of Hᵀ, while a plain streaming read of the same tile shape reaches 7.2 TB/s
// (profiles/r02/probes/stream_probe*.log).
//
// Layout: one 4-wave workgroup per CU, one wave per SIMD (up to 512 VGPRs); every wave owns its own
// 16-sample tiles gw + NW·i (gw = 4·blockIdx + wave, NW = 4·gridDim) and never waits for another
// wave inside an iteration.  Lane l = (sample s = l / 4, quarter q = l % 4); q owns features
// [21q, 21q + 21) (q = 3: 18 real features + 3 zero-Hᵀ pads).
//  * X: PD tiles (5184 B each) in flight per wave in registers (6 × 16 B per lane, the 6th for
//    lanes 0-3 only), staged to the wave's private LDS slot (in-order LDS: no barrier) and read
//    back per lane along its sample row (x kept in 21 VGPRs from phase 1 to phase 3).
//  * Hᵀ: the lane's 21 × 4 fp32 values and its HHᵀ row (fp64) live in VGPRs for the whole
//    iteration (reloaded after each basis update) — no Hᵀ read per tile.
//  * phase 1 (num = x·Hᵀ, SK:543): packed fp32 chains of 7 features folded into fp64 (the sl
//    arithmetic), then a DPP reduce-scatter inside the quad: lane q ends with num[s][q].
//  * phase 2 (SK:553-629): the fp64 update of w[s][q] against the LDS-resident W (each wave's tiles
//    stay in LDS for the whole launch), w' gathered back to the quad by DPP broadcasts.
//  * phase 3 (A += w'ᵀx, B += w'ᵀw', SK:639-640): packed fp32 accumulators per lane over the
//    iteration; at its end a DPP / permlane-swap butterfly over the 16 sample lanes of each q,
//    then the four waves' sums combined in fp64 in a fixed order -> the workgroup's partial row.
//  * the in-launch reduction (tickets, group / top combiners, flag), the basis update in every
//    workgroup and the optional cross-rank exchange are those of mu_iter_sl_kernel.
// ------------------------------------------------------------------------------------------------
namespace wt {
constexpr int F = 81;
constexpr int NWV = 4;                  // waves per workgroup (one per SIMD)
typedef float f2 __attribute__((ext_vector_type(2)));

// geometry of the wave tile for k = KK components: NL = KK lanes per sample (lane l = NL·s + e),
// TSW = 64 / NL samples per tile, NQ features per lane (e owns [NQ·e, NQ·e + NQ); the lanes past F
// hold zero-Hᵀ pads)
template <int KK>
struct Geo {
  static constexpr int K = KK, NL = KK, TSW = 64 / KK, V = F + KK, NOUT = KK * V;
  static constexpr int NQ = (F + KK - 1) / KK;              // 21 (k = 4), 11 (k = 8)
  static constexpr int XBW = TSW * F * 4;                   // 5184 / 2592 B of X per tile
  static constexpr int NCHW = XBW / 16;                     // 324 / 162 chunks
  static constexpr int PFW = (NCHW + 63) / 64;              // 6 / 3 loads per lane
  static constexpr int LASTL = NCHW - 64 * (PFW - 1);       // lanes of the last load: 4 / 34
  // phase 1 reads NQ features from lane e's first one, so the last sample's last lane runs OVR
  // floats past the tile (features >= F, zero Hᵀ): they must be finite — zeros kept in the slot
  static constexpr int OVR = (TSW - 1) * F + NQ * NL - XBW / 4;  // 3 (k = 4), 7 (k = 8)
  static constexpr int PADB = (OVR * 4 + 15) / 16 * 16;          // 16 / 32 zero bytes
  static constexpr int XSTR = XBW + PADB;                        // staging stride
  static constexpr int WBW = TSW * KK * 4;                  // 256 B of W per tile
  static constexpr int NACC = NQ * KK + KK;                 // fp32 accumulators per lane
  // LDS carve (bytes)
  static constexpr int L_STG = 0;                                       // [NWV][XSTR]
  static constexpr int L_WSTG = L_STG + NWV * XSTR;                     // streamed W: [NWV][WBW]
  static constexpr int L_RED = (L_WSTG + NWV * WBW + 15) / 16 * 16;     // [NWV][NL][NACC] fp32
  static constexpr int L_H = (L_RED + NWV * NL * NACC * 4 + 15) / 16 * 16;  // H fp64 [K][F]
  static constexpr int L_AB = L_H + KK * F * 8;                         // AB fp64 [K][V] (+ the loss)
  static constexpr int L_HT = L_AB + (NOUT + 2) * 8;                    // Hᵀ fp32 [NL·NQ][K]
  static constexpr int L_HHT = L_HT + NL * NQ * KK * 4;                 // HHᵀ fp64 [K][K]
  static constexpr int L_FLAG = L_HHT + KK * KK * 8;                    // 8 ints
  static constexpr int L_LOSS = L_FLAG + 32;                            // [NWV] wave loss sums, init, prev
  static constexpr int L_WRES = (L_LOSS + 8 * 8 + 15) / 16 * 16;        // [NWV][nbt_max][WBW]
  static_assert(NCHW * 16 == XBW && XBW % 16 == 0, "tiles are whole 16-byte chunks");
  static_assert(OVR >= 0 && PADB / 4 <= 64, "one zero float per lane covers the overrun");
  static_assert(NOUT <= 3 * NT, "three accumulator outputs per thread at most");
  static_assert(NOUT * 8 >= NWV * 64 * 4, "the prologue's dummy stores stay inside the partial row");
};

template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xFFFFFFFFll), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
// the value of lane l ^ 16 / l ^ 32 (v_permlane16/32_swap: lanes 32-63 of the first operand trade
// with lanes 0-31 of the second, resp. the odd 16-lane rows of the first with the even rows of the
// second; with both operands v, the first result holds l ^ 32 in the upper half / l ^ 16 in the odd
// rows, the second in the lower half / the even rows)
__device__ __forceinline__ double lane_xor16(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const bool odd = (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 16) != 0;
  return __hiloint2double(odd ? (int)b[0] : (int)b[1], odd ? (int)a[0] : (int)a[1]);
}
__device__ __forceinline__ double lane_xor32(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const bool up = (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 32) != 0;
  return __hiloint2double(up ? (int)b[0] : (int)b[1], up ? (int)a[0] : (int)a[1]);
}

// v summed over the lanes l' ≡ l (mod NL) of the wave (every lane gets its class's sum)
template <int NL>
__device__ __forceinline__ float sum_over_samples(float v) {
  if (NL == 4) v += dppf<0x124>(v);  // row_ror:4
  v += dppf<0x128>(v);               // row_ror:8
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // + lane ^ 16
  auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r2[0]) + __uint_as_float(r2[1]);  // + lane ^ 32
}

// Reduce-scatter of N per-lane floats over the lanes l' ≡ l (mod NL) (round 6): two permlane swap
// levels halve the values each (permlane32_swap(x, y): the lower half-wave ends with x's pair sum,
// the upper with y's; permlane16_swap likewise for even / odd 16-lane rows) — one swap and one add
// per PAIR of values, where the all-reduce form spends two of each per value — and the samples
// left inside a row are summed by DPP row rotations (ror 4 and 8 at NL = 4, ror 8 at NL = 8).
// On return v[0 .. N/4) of every lane of row r = l / 16 hold the totals of values
// j0 + [0, N/4) with j0 = (N/2)·(r >> 1) + (N/4)·(r & 1) (the same in the row's lanes of one class).
template <int NL, int N>
__device__ __forceinline__ void scatter_over_samples(float (&v)[N]) {
  static_assert(N % 4 == 0 && (NL == 4 || NL == 8), "four quarters of the values, 4 or 8 lanes per sample");
#pragma unroll
  for (int j = 0; j < N / 2; ++j) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j + N / 2]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int j = 0; j < N / 4; ++j) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[j]), __float_as_uint(v[j + N / 4]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int j = 0; j < N / 4; ++j) {
    if (NL == 4) v[j] += dppf<0x124>(v[j]);  // row_ror:4
    v[j] += dppf<0x128>(v[j]);               // row_ror:8
  }
}

// v summed over the 16 lanes of its row (every lane gets the row's sum)
__device__ __forceinline__ float sum_over_row16(float v) {
  v += dppf<0x128>(v);  // row_ror:8
  v += dppf<0x124>(v);  // row_ror:4
  v += dppf<0x122>(v);  // row_ror:2
  return v + dppf<0x121>(v);  // row_ror:1
}

// The X (and streamed W) prefetch lives in AGPRs and never touches a VGPR: inline-asm loads into
// AGPR tuples, an asm wait naming them "+a", and asm ds_write_b128 straight from the AGPRs into
// the staging slot (cdna_hip_programming.md §5.7 item 1, form ii).  Two reasons: (1) hipcc's own
// counted waits for compiler-issued loads degrade to vmcnt(0) at this loop's header (one tile in
// flight instead of PD), and (2) under this kernel's VGPR pressure hipcc parks VGPR-resident
// prefetch registers in AGPRs, copying them before the data has landed.  VMEM operations retire
// in issue order, so before staging set k, vmcnt(L·(PD-1)) (L loads per set) leaves exactly the
// PD-1 younger sets in flight; compiler-issued memory operations in between only make it stricter.
#ifdef CNMF_X_PLAIN
#define WT_LD "global_load_dwordx4 %0, %1, off"
#else
#define WT_LD "global_load_dwordx4 %0, %1, off nt"
#endif
__device__ __forceinline__ void ld16(u32x4& r, const unsigned char* p) {
  asm volatile(WT_LD : "=a"(r) : "v"(p) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N, int C>
__device__ __forceinline__ void wait_set(u32x4 (&pf)[C]) {
  static_assert(N >= 0 && N <= 63, "s_waitcnt vmcnt is a 6-bit field: a deeper prefetch cannot be counted");
  if constexpr (C == 7)
    asm volatile("s_waitcnt vmcnt(%7)"
                 : "+a"(pf[0]), "+a"(pf[1]), "+a"(pf[2]), "+a"(pf[3]), "+a"(pf[4]), "+a"(pf[5]), "+a"(pf[6])
                 : "n"(N) : "memory");
  else if constexpr (C == 6)
    asm volatile("s_waitcnt vmcnt(%6)"
                 : "+a"(pf[0]), "+a"(pf[1]), "+a"(pf[2]), "+a"(pf[3]), "+a"(pf[4]), "+a"(pf[5])
                 : "n"(N) : "memory");
  else if constexpr (C == 4)
    asm volatile("s_waitcnt vmcnt(%4)" : "+a"(pf[0]), "+a"(pf[1]), "+a"(pf[2]), "+a"(pf[3]) : "n"(N) : "memory");
  else if constexpr (C == 3)
    asm volatile("s_waitcnt vmcnt(%3)" : "+a"(pf[0]), "+a"(pf[1]), "+a"(pf[2]) : "n"(N) : "memory");
  else
    static_assert(C == 3 || C == 4 || C == 6 || C == 7, "prefetch set size");
}
template <int OFF>
__device__ __forceinline__ void st16(unsigned addr, const u32x4& v) {
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "a"(v), "i"(OFF) : "memory");
}
template <int OFF, int U>
__device__ __forceinline__ void stage_rec(unsigned addr, const u32x4* pf) {
  st16<OFF>(addr, pf[0]);
  if constexpr (U > 1) stage_rec<OFF + 1024, U - 1>(addr, pf + 1);
}
}  // namespace wt

// sum of `cnt` rows (m0, m0 + step, ...) of NOUT doubles each, in row order, sc1 loads (the NOUT-
// generic form of sum_rows_sc1: up to three outputs per thread, their row batches in flight together)
template <int NOUT>
__device__ __forceinline__ void sum_rows_n(const double* rows, int m0, int step, int cnt, double* lds_out,
                                           double* g_out, int t) {
  constexpr int U = (NOUT + NT - 1) / NT;
  constexpr int RB = U == 1 ? 16 : (U == 2 ? 16 : 8);
  int o[U];
  double v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    o[u] = t + NT * u < NOUT ? t + NT * u : t;
    v[u] = 0.0;
  }
  for (int m = 0; m < cnt; m += RB) {
    double x[RB][U];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int row = m0 + min(m + r, cnt - 1) * step;
#pragma unroll
      for (int u = 0; u < U; ++u) x[r][u] = ld_sc1(rows + (size_t)row * NOUT + o[u]);
    }
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] += m + r < cnt ? x[r][u] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (t + NT * u < NOUT) {
      if (lds_out) lds_out[o[u]] = v[u];
      st_sc1(g_out + o[u], v[u]);
    }
}

// 16-byte agent-scope (sc1) loads and stores: the valid-forms table's first row allows 16-B sc1
// stores and loads on both sides of a hand-off (MI355X_MICROARCH.md); one instruction per two doubles
// where sum_rows_n moved 8 bytes per lane (round 6: the guide's 8-B accesses run at 0.54-0.70x the
// 16-B rate, and the tail's combines were latency-bound on those loads, profiles/r06/tree/)
__device__ __forceinline__ void ld16_sc1(u32x4& r, const double* p) {
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(r) : "v"(p) : "memory");
}
__device__ __forceinline__ void st16_sc1v(double* p, double v0, double v1) {
  const u32x4 v = u32x4{(unsigned)__double2loint(v0), (unsigned)__double2hiint(v0), (unsigned)__double2loint(v1),
                        (unsigned)__double2hiint(v1)};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st16_plain(double* p, double v0, double v1) {
  const u32x4 v = u32x4{(unsigned)__double2loint(v0), (unsigned)__double2hiint(v0), (unsigned)__double2loint(v1),
                        (unsigned)__double2hiint(v1)};
  asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ double lo_d(const u32x4& r) { return __hiloint2double((int)r[1], (int)r[0]); }
__device__ __forceinline__ double hi_d(const u32x4& r) { return __hiloint2double((int)r[3], (int)r[2]); }
template <int N>
__device__ __forceinline__ void wait8(u32x4 (&x)[8]) {
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
               : "n"(N) : "memory");
}
// sum_rows_n for an even NOUT with 16-byte sc1 loads: thread t owns the chunks (doubles 2c, 2c + 1)
// c = t (and c = t + NT when NOUT / 2 > NT: k = 8) of every row and adds the rows in row order
// (0.0 + r0 + r1 + ...: the same operations, the same bits as sum_rows_n); 16 loads in flight per
// batch (one chunk: 16 rows, two waits of 8 in issue order; two chunks: 8 rows each); the result
// goes to lds_out (optional) and, with 16-byte sc1 stores, to g_out
template <int NOUT>
__device__ __forceinline__ void sum_rows_v(const double* rows, int m0, int step, int cnt, double* lds_out,
                                           double* g_out, int t) {
  static_assert(NOUT % 2 == 0 && NOUT / 2 <= 2 * NT, "one or two 16-byte chunks per thread");
  constexpr int NCH = NOUT / 2, UC = NCH > NT ? 2 : 1;
  const int c0 = t < NCH ? t : NCH - 1;                    // threads past the row re-load its last chunk
  const int c1 = t + NT < NCH ? t + NT : NCH - 1;          // (never stored)
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
  if constexpr (UC == 1) {
    for (int m = 0; m < cnt; m += 16) {
      u32x4 xa[8], xb[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) ld16_sc1(xa[r], rows + (size_t)(m0 + min(m + r, cnt - 1) * step) * NOUT + 2 * c0);
#pragma unroll
      for (int r = 0; r < 8; ++r) ld16_sc1(xb[r], rows + (size_t)(m0 + min(m + 8 + r, cnt - 1) * step) * NOUT + 2 * c0);
      wait8<8>(xa);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        v0 += m + r < cnt ? lo_d(xa[r]) : 0.0;
        v1 += m + r < cnt ? hi_d(xa[r]) : 0.0;
      }
      wait8<0>(xb);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        v0 += m + 8 + r < cnt ? lo_d(xb[r]) : 0.0;
        v1 += m + 8 + r < cnt ? hi_d(xb[r]) : 0.0;
      }
    }
  } else {
    for (int m = 0; m < cnt; m += 8) {
      u32x4 xa[8], xb[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const size_t row = (size_t)(m0 + min(m + r, cnt - 1) * step) * NOUT;
        ld16_sc1(xa[r], rows + row + 2 * c0);
        ld16_sc1(xb[r], rows + row + 2 * c1);
      }
      wait8<0>(xa);  // (both arrays' loads are interleaved: wait for all)
      wait8<0>(xb);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        v0 += m + r < cnt ? lo_d(xa[r]) : 0.0;
        v1 += m + r < cnt ? hi_d(xa[r]) : 0.0;
        v2 += m + r < cnt ? lo_d(xb[r]) : 0.0;
        v3 += m + r < cnt ? hi_d(xb[r]) : 0.0;
      }
    }
  }
  if (t < NCH) {
    if (lds_out) {
      lds_out[2 * t] = v0;
      lds_out[2 * t + 1] = v1;
    }
    st16_sc1v(g_out + 2 * t, v0, v1);
  }
  if (UC == 2 && t + NT < NCH) {
    if (lds_out) {
      lds_out[2 * (t + NT)] = v2;
      lds_out[2 * (t + NT) + 1] = v3;
    }
    st16_sc1v(g_out + 2 * (t + NT), v2, v3);
  }
}

// the cross-rank all-reduce of AB inside a persistent launch (xchg_allreduce_ab's protocol,
// generic in the accumulator count NOUT; slot stride 2·NOUT words)
template <int NOUT>
__device__ __forceinline__ void xchg_allreduce_n(uint64_t* xctl, double* AB, double* sAB, uint32_t* err, int it, int t) {
  constexpr int U = (NOUT + NT - 1) / NT;
  const int xrank = (int)__hip_atomic_load(xctl + XC_RANK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int xworld = (int)__hip_atomic_load(xctl + XC_WORLD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t gen =
      (uint32_t)__hip_atomic_load(xctl + XC_GEN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (uint32_t)it + 1u;
  auto peer = [&](int r) {
    return reinterpret_cast<uint64_t*>(__hip_atomic_load(xctl + XC_PEERS + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  };
  TL_X(it, 0);
  const size_t slot = 2 * (size_t)NOUT;
  const size_t par = (size_t)(gen & 1u) * xworld * slot;
  int o[U];
#pragma unroll
  for (int u = 0; u < U; ++u) o[u] = t + NT * u < NOUT ? t + NT * u : t;
  {
    const bool bad = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    const uint64_t tag = (uint64_t)(bad ? sl::XPOISON : gen) << 32;
    for (int pr = 0; pr < xworld; ++pr) {
      uint64_t* dst = peer(pr) + par + (size_t)xrank * slot;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (t + NT * u < NOUT) {
          const uint64_t bv = (uint64_t)__double_as_longlong(sAB[o[u]]);
          __hip_atomic_store(dst + 2 * o[u], tag | (bv & 0xFFFFFFFFull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(dst + 2 * o[u] + 1, tag | (bv >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
  }
  TL_X(it, 1);
  const uint64_t* mine = peer(xrank) + par;
  double v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = 0.0;
  constexpr int QB = 4;  // ranks polled per round (their loads in flight together)
  for (int q0 = 0; q0 < xworld; q0 += QB) {
    uint64_t w[QB][2 * U];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
      const uint32_t ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // same batch
#pragma unroll
      for (int j = 0; j < QB; ++j) {
        const uint64_t* src = mine + (size_t)min(q0 + j, xworld - 1) * slot;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          w[j][2 * u] = __hip_atomic_load(src + 2 * o[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          w[j][2 * u + 1] = __hip_atomic_load(src + 2 * o[u] + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      bool ok = true, poison = false;
#pragma unroll
      for (int j = 0; j < QB; ++j)
#pragma unroll
        for (int m = 0; m < 2 * U; ++m) {
          const uint32_t tg = (uint32_t)(w[j][m] >> 32);
          ok = ok && tg == gen;
          poison = poison || tg == sl::XPOISON;
        }
      if (ok) break;
      if (poison) {
        __hip_atomic_store(err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      if (ev != 0u) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > sl::SPIN_TIMEOUT) {
        __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int j = 0; j < QB; ++j)
      if (q0 + j < xworld)  // rank order
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[u] += __longlong_as_double((long long)((w[j][2 * u + 1] << 32) | (w[j][2 * u] & 0xFFFFFFFFull)));
  }
  TL_X(it, 2);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (t + NT * u < NOUT) {
      sAB[o[u]] = v[u];
      st_sc1(AB + o[u], v[u]);
    }
  TL_X(it, 3);
}

// HHᵀ (fp64) from the fp64 H in LDS: NT / K² consecutive threads per entry (16 at k = 4: one DPP row;
// 4 at k = 8: a quad), each a strided part of the F products, then a fixed DPP butterfly over the
// group (xor 1, xor 2 by quad_perm; at 16 the half-row and row mirrors) — register moves where the
// round-5 xor tree went through the LDS crossbar (ds_bpermute, a dependent round trip per level).
// Every entry takes the same operations in the same order, and HHᵀ[j][m] / HHᵀ[m][j] are the same
// products, so it stays exactly symmetric.  Caller synchronises.
template <int KK, class G = wt::Geo<KK>>
__device__ __forceinline__ void wt_hht(unsigned char* smem, int t) {
  const double* sH = reinterpret_cast<const double*>(smem + G::L_H);
  double* sHHt = reinterpret_cast<double*>(smem + G::L_HHT);
  constexpr int NE = KK * KK, TPE = NT / NE;
  static_assert(TPE * NE == NT && (TPE == 4 || TPE == 16), "threads per HHᵀ entry: a quad or a DPP row");
  const int en = t / TPE, part = t - en * TPE;
  const int j = en / KK, m = en - (en / KK) * KK;
  // the strided products with a compile-time trip count: every LDS read of the row pair issued
  // before the first FMA (a runtime loop waited on each iteration's reads in turn)
  constexpr int NF = (wt::F + TPE - 1) / TPE;
  double hj[NF], hm[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int f = part + TPE * i < wt::F ? part + TPE * i : wt::F - 1;
    hj[i] = sH[j * wt::F + f];
    hm[i] = sH[m * wt::F + f];
  }
  double v = 0.0;
#pragma unroll
  for (int i = 0; i < NF; ++i)
    if (part + TPE * i < wt::F) v = fma(hj[i], hm[i], v);
  v += wt::dpp64<0xB1>(v);  // quad_perm [1,0,3,2]
  v += wt::dpp64<0x4E>(v);  // quad_perm [2,3,0,1]
  if constexpr (TPE == 16) {
    v += wt::dpp64<0x141>(v);  // row_half_mirror: the other quad of the half-row
    v += wt::dpp64<0x140>(v);  // row_mirror: the other half-row
  }
  if (part == 0) sHHt[en] = v;
}
// Hᵀ (fp32, the lanes' feature blocks, rows >= F zero) and HHᵀ from the fp64 H in LDS — sl_derive_basis
// for k = KK
template <int KK, class G = wt::Geo<KK>>
__device__ __forceinline__ void wt_derive_basis(unsigned char* smem, int t) {
  const double* sH = reinterpret_cast<const double*>(smem + G::L_H);
  float* sHt = reinterpret_cast<float*>(smem + G::L_HT);
  for (int e = t; e < G::NL * G::NQ * KK; e += NT) {
    const int f = e / KK;
    const int j = e - f * KK;
    sHt[e] = f < wt::F ? (float)sH[j * wt::F + f] : 0.f;
  }
  wt_hht<KK, G>(smem, t);
  __syncthreads();
}
// H <- H·(WᵀX / ((WᵀW)·H (+l1)(+l2·H))) on the fp64 H in LDS from AB in LDS (SK:634-728) —
// sl_update_basis for k = KK.  Round 6: the quotient as div_nr (v_rcp_f64 + one Newton step, the
// W-update's arithmetic) and the new Hᵀ written with the new H (its pad rows stay zero), then HHᵀ
template <int KK, class G = wt::Geo<KK>>
__device__ __forceinline__ void wt_update_basis(unsigned char* smem, int t, double l1, double l2) {
  constexpr int KF = KK * wt::F;
  constexpr int U = (KF + NT - 1) / NT;
  double* sH = reinterpret_cast<double*>(smem + G::L_H);
  float* sHt = reinterpret_cast<float*>(smem + G::L_HT);
  const double* sAB = reinterpret_cast<const double*>(smem + G::L_AB);
  double hn[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = t + NT * u;
    hn[u] = 0.0;
    if (e < KF) {
      const int j = e / wt::F;
      const int f = e - j * wt::F;
      const double h = sH[e];
      const double num = sAB[j * G::V + f];                                      // (WᵀX)[j][f], SK:639
      double den = 0.0;                                                          // ((WᵀW)·H)[j][f], SK:640
      for (int m = 0; m < KK; ++m) den = fma(sAB[j * G::V + wt::F + m], sH[m * wt::F + f], den);
      if (l1 > 0.0) den += l1;                                                   // SK:702-703
      if (l2 > 0.0) den = den + l2 * h;                                          // SK:704-705
      if (den == 0.0) den = EPS32;                                               // SK:706
      hn[u] = h * div_nr(num, den);                                              // SK:722-726
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = t + NT * u;
    if (e < KF) {
      const int j = e / wt::F;
      const int f = e - j * wt::F;
      sH[e] = hn[u];
      sHt[f * KK + j] = (float)hn[u];
    }
  }
  // Hᵀ's pad rows (features >= F, read by the lanes past F): zero (a launch that starts with the
  // pending update, apply_first, has not run wt_derive_basis)
  for (int e = wt::F * KK + t; e < G::NL * G::NQ * KK; e += NT) sHt[e] = 0.f;
  __syncthreads();
  wt_hht<KK, G>(smem, t);
  __syncthreads();
}

// The round-5 forms of wt_derive_basis / wt_update_basis (xor-shuffle HHᵀ tree, IEEE division), kept
// for k = 8: the round-6 end of iteration measured 3.5 % slower on cfg3's k = 8 shard (the streaming
// body's schedule, not the tail; profiles/r06/tree/), so that kernel keeps the round-5 tail.
// Hᵀ (fp32, the lanes' feature blocks, rows >= F zero) and HHᵀ (fp64; lanes over f, fixed shuffle
// tree) from the fp64 H in LDS — sl_derive_basis for k = KK
template <int KK, class G = wt::Geo<KK>>
__device__ __forceinline__ void wt_derive_basis_r5(unsigned char* smem, int t) {
  const double* sH = reinterpret_cast<const double*>(smem + G::L_H);
  float* sHt = reinterpret_cast<float*>(smem + G::L_HT);
  double* sHHt = reinterpret_cast<double*>(smem + G::L_HHT);
  for (int e = t; e < G::NL * G::NQ * KK; e += NT) {
    const int f = e / KK;
    const int j = e - f * KK;
    sHt[e] = f < wt::F ? (float)sH[j * wt::F + f] : 0.f;
  }
  // HHᵀ: NT / K² consecutive threads per entry (16 at k = 4, 4 at k = 8), each a strided part of the
  // F products, then a fixed xor tree over the group (every entry in the same order; HHᵀ[j][m] and
  // HHᵀ[m][j] are the same products, so it stays exactly symmetric)
  constexpr int NE = KK * KK, TPE = NT / NE;
  static_assert(TPE * NE == NT && (TPE & (TPE - 1)) == 0, "threads per HHᵀ entry: a power of two");
  const int en = t / TPE, part = t - en * TPE;
  const int j = en / KK, m = en - (en / KK) * KK;
  double v = 0.0;
  for (int f = part; f < wt::F; f += TPE) v = fma(sH[j * wt::F + f], sH[m * wt::F + f], v);
#pragma unroll
  for (int o = TPE / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (part == 0) sHHt[en] = v;
  __syncthreads();
}
// H <- H·(WᵀX / ((WᵀW)·H (+l1)(+l2·H))) on the fp64 H in LDS from AB in LDS (SK:634-728) —
// sl_update_basis for k = KK
template <int KK, class G = wt::Geo<KK>>
__device__ __forceinline__ void wt_update_basis_r5(unsigned char* smem, int t, double l1, double l2) {
  constexpr int KF = KK * wt::F;
  constexpr int U = (KF + NT - 1) / NT;
  double* sH = reinterpret_cast<double*>(smem + G::L_H);
  const double* sAB = reinterpret_cast<const double*>(smem + G::L_AB);
  double hn[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = t + NT * u;
    hn[u] = 0.0;
    if (e < KF) {
      const int j = e / wt::F;
      const int f = e - j * wt::F;
      const double h = sH[e];
      const double num = sAB[j * G::V + f];                                      // (WᵀX)[j][f], SK:639
      double den = 0.0;                                                          // ((WᵀW)·H)[j][f], SK:640
      for (int m = 0; m < KK; ++m) den = fma(sAB[j * G::V + wt::F + m], sH[m * wt::F + f], den);
      if (l1 > 0.0) den += l1;                                                   // SK:702-703
      if (l2 > 0.0) den = den + l2 * h;                                          // SK:704-705
      if (den == 0.0) den = EPS32;                                               // SK:706
      hn[u] = h * (num / den);                                                   // SK:722-726
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (t + NT * u < KF) sH[t + NT * u] = hn[u];
  __syncthreads();
  wt_derive_basis_r5<KK, G>(smem, t);
}

// TOL: the tolerance test of SK:872-884 on the device.  In iteration g + 1 (g = it0 + it, g % 10 ==
// 0) each lane also accumulates ‖x − w·H‖² of the state AFTER g iterations (x, the old w and H are
// all in registers then: fp32 residual per element, fp64 sums per tile), carried as one more
// column of the partial rows (NOUT + 1) and reduced / exchanged with [WᵀX | WᵀW]; the top combiner
// applies the relative-decrease test.  On a stop it publishes the flag with FLAG_STOP and every
// workgroup leaves with the state after g iterations: H (not updated), W as it was before this
// iteration's update — written to W itself in the loss iterations when W is resident in LDS, else to
// the snapshot buffer (TC_WSNAP; the host copies it) — so n_iter = g as in sklearn.
template <int KK, bool WRES, int PD, bool MULTI = false, bool TOL = false>
__global__ __launch_bounds__(NT, 1) void mu_iter_wt_kernel(PersistArgs a) {
  using namespace wt;
  using G_ = Geo<KK>;
  constexpr int NL = G_::NL, TSW = G_::TSW, NQ = G_::NQ, V = G_::V, NOUT = G_::NOUT;
  constexpr int NOUTT = NOUT + (TOL ? 1 : 0);  // partial-row width: + the loss of the checked state
  // row stride of the partial / group rows and AB: even, so that every row is 16-byte chunks (round 6:
  // 16-byte sc1 hand-offs; TOL's odd NOUTT + a zero pad — cnmf_mu_fit_tol's rows of k(F+k) + 2)
  // k = 8 keeps the round-5 tail (8-byte hand-offs, the round-5 basis update; see wt_update_basis_r5)
  constexpr bool R6 = KK == 4;
  constexpr int RS = R6 ? (NOUTT + 1) & ~1 : NOUTT;
  constexpr int XBW = G_::XBW, XSTR = G_::XSTR, WBW = G_::WBW, NACC = G_::NACC;
  constexpr int PFW = G_::PFW, LASTL = G_::LASTL;
  constexpr int PFS = PFW + (WRES ? 0 : 1);  // loads per prefetch set (+ the W tile when streamed)
  // stores per body: W streamed — its W tile, and TOL's snapshot of the checked state's W (a resident
  // W keeps that snapshot in LDS: no store, so the counted waits are the plain kernel's)
  constexpr int NSTB = (WRES ? 0 : 1) + (TOL && !WRES ? 1 : 0);
  constexpr int KP = KK / 2;                 // component pairs
  // the PD prefetch sets live in AGPRs (4 per load) next to the kernel's own registers: past a
  // budget the allocator spills them to scratch right behind their loads, i.e. before the data has
  // landed, and the staged tiles are stale (k = 8 streamed W at PD = 6: 96 AGPRs, all-NaN W at 2.5x
  // the time).  tools/kcheck.py checks the built library for exactly that; the
  // depths measured clean are allowed here (k = 8: PD <= 5, 80 AGPRs; k = 4: PD <= 4, 96)
  static_assert(4 * PD * PFS <= (KK == 8 ? 80 : 96), "prefetch depth past the measured AGPR budget");
  static_assert(PFS * (PD - 1) + NSTB * PD <= 63, "the counted wait's vmcnt is a 6-bit field");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int t = threadIdx.x;
  const int l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int s = l / NL, e = l % NL;
  const int b = blockIdx.x;
  const int G = gridDim.x;
  const int NW = NWV * G;
  const int gw = NWV * b + w;
  const int NG = a.n_groups;
  const int g = b % NG;
  const int gs = (G - g + NG - 1) / NG;
  const unsigned char* Xb = reinterpret_cast<const unsigned char*>(a.X);
  unsigned char* Wb = reinterpret_cast<unsigned char*>(a.W);
  const int nbt = (int)((a.n_tiles - gw + NW - 1) / NW);  // this wave's tiles per iteration
  const int nbt_max = (int)((a.n_tiles + NW - 1) / NW);
  unsigned char* stg = smem + G_::L_STG + w * XSTR;
  unsigned char* wstg = smem + G_::L_WSTG + w * WBW;  // streamed W: this wave's current tile
  // W streamed: its first nres tiles per wave resident all the same (the LDS the plan has left; round
  // 5): their W loads re-load an X chunk (the counted waits see the same loads) and their stores go
  // to the dummy word (the same stores), the rest streams
  const int nres = WRES ? 0 : __builtin_amdgcn_readfirstlane(a.n_static);
  float* wres = reinterpret_cast<float*>(smem + G_::L_WRES + (size_t)w * (WRES ? nbt_max : nres) * WBW);  // [i][TSW][K]
  float* red = reinterpret_cast<float*>(smem + G_::L_RED);
  double* sH = reinterpret_cast<double*>(smem + G_::L_H);
  double* sAB = reinterpret_cast<double*>(smem + G_::L_AB);
  int* sFlag = reinterpret_cast<int*>(smem + G_::L_FLAG);
  double* sLoss = reinterpret_cast<double*>(smem + G_::L_LOSS);
  // TOL: the launch's first global iteration, the snapshot buffer (streamed W)
  const int it0 = TOL ? (int)ld_sc1(a.tolctl + TC_IT0) : 0;
  // TOL: every workgroup tracks the test's error at init and previous error itself (sLoss[4], [5]),
  // so the decision of the iteration's top combiner reads no state another workgroup wrote
  const double tolv = TOL ? ld_sc1(a.tolctl + TC_TOL) : 0.0;
  if (TOL && t == 0) {
    sLoss[4] = ld_sc1(a.tolctl + TC_INIT);
    sLoss[5] = ld_sc1(a.tolctl + TC_PREV);
  }
  float* wsnap = (TOL && !WRES)
                     ? reinterpret_cast<float*>(__double_as_longlong(ld_sc1(a.tolctl + TC_WSNAP)))
                     : nullptr;
  // TOL with W resident: the W of the state a loss iteration checks, this wave's tiles [i][TSW][K],
  // after the four waves' resident W (the host sizes the LDS for both)
  float* wsnapl = (TOL && WRES) ? reinterpret_cast<float*>(smem + G_::L_WRES + (size_t)(NWV + w) * nbt_max * WBW)
                                : nullptr;
  double lossacc = 0.0;  // this lane's ‖x − w·H‖² over the iteration's tiles (loss iterations)
  uint32_t* cnt_group = a.cnt + CNT_GROUP0 + 32 * g;
  uint32_t* cnt_top = a.cnt + CNT_TOP;
  uint32_t* flag = a.cnt + CNT_FLAG;
  uint32_t* err = a.cnt + CNT_ERR;

  // ---- the basis for the first iteration, the staging pads, this wave's W tiles (W resident)
  const bool l2rows = R6 && a.l2rows != 0;
  if (t == 0) {  // the XCC this workgroup runs on, into the table (read once, after iteration 0)
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    sFlag[4] = 0;  // partial rows write-through until the group's placement has been checked
    sFlag[5] = (int)(xcc & 0xFu) + 1;
    if (l2rows) __hip_atomic_store(a.cnt + CNT_XCC0 + b, (xcc & 0xFu) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int i = t; i < KK * F; i += NT) sH[i] = a.H64[i];
  if (a.apply_first)
    for (int i = t; i < NOUT; i += NT) sAB[i] = a.AB[i];
  if (l < G_::PADB / 4) reinterpret_cast<float*>(stg + XBW)[l] = 0.f;
  {
    const int nw = WRES ? nbt : min(nres, nbt);
    for (int c = l; c < nw * (WBW / 16); c += 64) {
      const int i = c / (WBW / 16), ch = c - i * (WBW / 16);
      *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned char*>(wres) + i * WBW + 16 * ch) =
          *reinterpret_cast<const u32x4*>(Wb + (size_t)(gw + (int64_t)NW * i) * WBW + 16 * ch);
    }
  }
  __syncthreads();
  if (a.apply_first) {
    if constexpr (R6) wt_update_basis<KK>(smem, t, a.l1H, a.l2H);
    else wt_update_basis_r5<KK>(smem, t, a.l1H, a.l2H);
  } else {
    if constexpr (R6) wt_derive_basis<KK>(smem, t);
    else wt_derive_basis_r5<KK>(smem, t);
  }

  // the lane's Hᵀ (fp32 component pairs of each of its NQ features) and HHᵀ row e
  f2 hp[NQ][KP];
  double hh[KK];
  f2 hh32[KP];  // k = 8: the HHᵀ row in fp32 pairs for the denominator
  auto load_basis = [&]() {
    const float* sHt = reinterpret_cast<const float*>(smem + G_::L_HT);
    const double* sHHt = reinterpret_cast<const double*>(smem + G_::L_HHT);
#pragma unroll
    for (int c = 0; c < NQ; ++c)
#pragma unroll
      for (int p4 = 0; p4 < KK / 4; ++p4) {
        const float4 h = *reinterpret_cast<const float4*>(sHt + (NQ * e + c) * KK + 4 * p4);
        hp[c][2 * p4] = f2{h.x, h.y};
        hp[c][2 * p4 + 1] = f2{h.z, h.w};
      }
#pragma unroll
    for (int m = 0; m < KK; ++m) hh[m] = sHHt[e * KK + m];
#pragma unroll
    for (int q = 0; q < KP; ++q) hh32[q] = f2{(float)hh[2 * q], (float)hh[2 * q + 1]};
  };
  load_basis();

  f2 acc[NQ][KP], accB[KP];
  auto zero_acc = [&]() {
#pragma unroll
    for (int c = 0; c < NQ; ++c)
#pragma unroll
      for (int p = 0; p < KP; ++p) acc[c][p] = f2{0.f, 0.f};
#pragma unroll
    for (int p = 0; p < KP; ++p) accB[p] = f2{0.f, 0.f};
  };
  zero_acc();

  // the tile's 16-byte chunks of this lane: l + 64u (u < PFW - 1) and, for lanes < LASTL, the last
  // (other lanes re-load chunk l: never staged; every lane issues the same loads), then the W tile
  // when streamed (lanes < 16; others re-load chunk l)
  auto prefetch = [&](u32x4 (&pf)[PFS], int64_t tile, int ti) {
#ifdef CNMF_DIAG_L2
    const unsigned char* xs = Xb + (size_t)(tile & 255) * XBW + 16 * l;
#else
    const unsigned char* xs = Xb + (size_t)tile * XBW + 16 * l;
#endif
#pragma unroll
    for (int u = 0; u < PFW - 1; ++u) ld16(pf[u], xs + 1024 * u);
    ld16(pf[PFW - 1], l < LASTL ? xs + 1024 * (PFW - 1) : xs);
    if (!WRES) ld16(pf[PFW], (l < WBW / 16 && ti >= nres) ? Wb + (size_t)tile * WBW + 16 * l : xs);
  };
  auto stage = [&](const u32x4 (&pf)[PFS]) {
    const unsigned addr = (unsigned)(uintptr_t)(stg + 16 * l);
    stage_rec<0, PFW - 1>(addr, pf);
    if (l < LASTL) st16<1024 * (PFW - 1)>(addr, pf[PFW - 1]);
    if (!WRES && l < WBW / 16) st16<0>((unsigned)(uintptr_t)(wstg + 16 * l), pf[PFW]);
  };

  const int total = a.n_iter * nbt;
  u32x4 pf[PD][PFS];
  // W streamed: after each of the first PD sets one dummy store (to this workgroup's partial row,
  // rewritten at the iteration's end), so that every set — the first PD too — has exactly PD stores
  // younger than it when its step waits (set q < PD: PD - q dummies, then the W stores of bodies
  // 0..q-1).  Counting PD stores that were never issued would let the set's last loads (the W tile)
  // still be in flight when it is staged.
  float* dummy = reinterpret_cast<float*>(a.partials + (size_t)b * RS) + 64 * w + l;
#pragma unroll
  for (int k = 0; k < PD; ++k) {
    prefetch(pf[k], gw + (int64_t)NW * k, k);  // the host keeps nbt > PD
#pragma unroll
    for (int d = 0; d < NSTB; ++d) asm volatile("global_store_dword %0, %1, off" ::"v"(dummy), "v"(0) : "memory");
  }
  // W streamed: a tile's W store (body x) must have retired before its next load is issued (the
  // prefetch at step x + nbt - PD); the step waits retire every operation older than the set they
  // wait for, which covers that store when nbt >= 2·PD + 1 (the host guarantees it)
  TL_START;

  bool alive = true;
  // position counters (wave-uniform, incremental: no division per tile): the tile being processed
  // (iteration cur_it, index cur_i) and the next one to prefetch (nx_i).  Every step stages its
  // register set and re-issues it unconditionally (past the launch's last position: the wave's
  // first tile again, never used), so the count of younger loads is the same on every path.
  int cur_i = 0, cur_it = 0, nx_i = PD;
  auto step = [&](u32x4 (&pfk)[PFS]) {
    // younger than this set's loads: the PD-1 later sets and the stores of the PD bodies since
    // (for the launch's first PD sets the prologue's dummy stores): with W streamed its W store, and
    // TOL the snapshot store every body issues (a loss iteration's W, else a dummy)
    wait_set<PFS * (PD - 1) + NSTB * PD, PFS>(pfk);
    stage(pfk);
    prefetch(pfk, gw + (int64_t)NW * nx_i, nx_i);
    if (++nx_i == nbt) nx_i = 0;
  };
  auto body = [&]() {
    const int it = cur_it, i = cur_i;
    if (++cur_i == nbt) {
      cur_i = 0;
      ++cur_it;
    }
    const bool last_it = it + 1 == a.n_iter;
#ifdef CNMF_TOL_NOLOSS  // timing-only diagnostic: the TOL kernel without its loss iterations (never stops)
    const bool loss_it = false;
#else
    const bool loss_it = TOL && ((it0 + it) % 10 == 0);  // check the state after it0 + it iterations
#endif
    const int64_t tile = gw + (int64_t)NW * i;
    // phase 2 first where it does not need x: the sample's W row and den = w·HHᵀ[e] with its refined
    // reciprocal (div_nr's v_rcp_f64 + Newton step, so w·num·r is div_nr's arithmetic) — their loads
    // and their ~15-deep dependent chain then overlap phase 1 instead of following the reduce-scatter
    // (round 5).  SK:553-629
    const bool wr = WRES || i < nres;  // this tile's W resident
    float* wt_ = wr ? wres + i * (TSW * KK) : reinterpret_cast<float*>(wstg);
    float wv[KK];
#pragma unroll
    for (int m4 = 0; m4 < KK / 4; ++m4) {
      const float4 v4 = *reinterpret_cast<const float4*>(wt_ + s * KK + 4 * m4);
      wv[4 * m4] = v4.x;
      wv[4 * m4 + 1] = v4.y;
      wv[4 * m4 + 2] = v4.z;
      wv[4 * m4 + 3] = v4.w;
    }
    const float wold32 = wt_[s * KK + e];
    const double wold = (double)wold32;
    double den = 0.0;
    if constexpr (KK == 8) {
      // den = w·HHᵀ[e] in packed fp32 (8 positive terms: no cancellation, ≤ 8 roundings), the
      // update itself in fp64
      f2 d2 = f2{0.f, 0.f};
#pragma unroll
      for (int q = 0; q < KP; ++q) d2 = __builtin_elementwise_fma(f2{wv[2 * q], wv[2 * q + 1]}, hh32[q], d2);
      den = (double)(d2.x + d2.y);
    } else {
#pragma unroll
      for (int m = 0; m < KK; ++m) den = fma((double)wv[m], hh[m], den);
    }
    if (a.l1W > 0.0) den += a.l1W;              // SK:616-617
    if (a.l2W > 0.0) den = den + a.l2W * wold;  // SK:618-619
    if (den == 0.0) den = EPS32;                // SK:620
    double rden = __builtin_amdgcn_rcp(den);
    rden = fma(rden, fma(-den, rden, 1.0), rden);
    // phase 1: x along the lane's row, packed fp32 chains of 7 features folded into fp64
    const float* xr = reinterpret_cast<const float*>(stg) + s * F + NQ * e;
    float xv[NQ];
#pragma unroll
    for (int c = 0; c < NQ; ++c) xv[c] = xr[c];
    double num;
    if constexpr (KK == 8) {
      // k = 8: ONE fp32 chain over the lane's 11 features, then the reduce-scatter over the
      // sample's 8 lanes in fp32 (3 adds per value; a chain of 11 + 3 roundings, below the 7-term
      // chains' error budget of §4), one DPP move per 32-bit value: level 1 pairs lane e with 7 - e
      // (row_half_mirror: the other half of components), then e ^ 2 and e ^ 1 (quad_perm)
      f2 ch[KP];
#pragma unroll
      for (int q = 0; q < KP; ++q) ch[q] = f2{0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NQ; ++c) {
        const f2 xx = f2{xv[c], xv[c]};
#pragma unroll
        for (int q = 0; q < KP; ++q) ch[q] = __builtin_elementwise_fma(xx, hp[c][q], ch[q]);
      }
      const bool b4 = (e & 4) != 0, b2 = (e & 2) != 0, b1 = (e & 1) != 0;
      f2 r[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const f2 keep = b4 ? ch[2 + m] : ch[m], send = b4 ? ch[m] : ch[2 + m];
        r[m] = keep + f2{dppf<0x141>(send.x), dppf<0x141>(send.y)};  // row_half_mirror
      }
      const f2 keep2 = b2 ? r[1] : r[0], send2 = b2 ? r[0] : r[1];
      const f2 t2 = keep2 + f2{dppf<0x4E>(send2.x), dppf<0x4E>(send2.y)};  // quad_perm [2,3,0,1]
      const float keep1 = b1 ? t2.y : t2.x, send1 = b1 ? t2.x : t2.y;
      num = (double)(keep1 + dppf<0xB1>(send1));  // quad_perm [1,0,3,2]
    } else {
      // k = 4: packed fp32 chains of 7 features folded into fp64, fp64 reduce-scatter over the
      // sample's 4 lanes
      double p[KK];
#pragma unroll
      for (int c0 = 0; c0 < NQ; c0 += 7) {
        f2 ch[KP];
#pragma unroll
        for (int q = 0; q < KP; ++q) ch[q] = f2{0.f, 0.f};
#pragma unroll
        for (int c = c0; c < (c0 + 7 < NQ ? c0 + 7 : NQ); ++c) {
          const f2 xx = f2{xv[c], xv[c]};
#pragma unroll
          for (int q = 0; q < KP; ++q) ch[q] = __builtin_elementwise_fma(xx, hp[c][q], ch[q]);
        }
#pragma unroll
        for (int q = 0; q < KP; ++q) {
          if (c0 == 0) {
            p[2 * q] = (double)ch[q].x;
            p[2 * q + 1] = (double)ch[q].y;
          } else {
            p[2 * q] += (double)ch[q].x;
            p[2 * q + 1] += (double)ch[q].y;
          }
        }
      }
      const bool b1 = (e & 1) != 0, b2 = (e & 2) != 0;
      double k2[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const double keep = b2 ? p[2 + m] : p[m], send = b2 ? p[m] : p[2 + m];
        k2[m] = keep + dpp64<0x4E>(send);  // quad_perm [2,3,0,1]
      }
      const double keep = b1 ? k2[1] : k2[0], send = b1 ? k2[0] : k2[1];
      num = keep + dpp64<0xB1>(send);  // quad_perm [1,0,3,2]
    }
    if constexpr (TOL && WRES) {
      // the W of the state a loss iteration checks, kept in LDS (written to HBM only on a stop)
      if (loss_it) wsnapl[i * (TSW * KK) + s * KK + e] = wold32;
    } else if constexpr (TOL) {
      // W streamed: the W of the checked state, ONE store per body in every iteration (the steps'
      // waits count it): a loss iteration stores the tile's W into the snapshot buffer, the others
      // the same value over the wave's first tile there, which the next loss iteration overwrites
      // (a stop happens only at the end of a loss iteration)
      const int64_t tsel = loss_it ? tile : (int64_t)gw;
      wsnap[(size_t)tsel * TSW * KK + l] = wold32;
    }
    if (loss_it) {
      // ‖x − w·H‖² of the state before this update, the lane's NQ features (the last lane's overrun
      // features past F belong to the next sample: masked)
      float l2 = 0.f;
#pragma unroll
      for (int c = 0; c < NQ; ++c) {
        f2 r2 = f2{0.f, 0.f};
#pragma unroll
        for (int q = 0; q < KP; ++q) r2 = __builtin_elementwise_fma(f2{wv[2 * q], wv[2 * q + 1]}, hp[c][q], r2);
        const float r = NQ * e + c < F ? xv[c] - (r2.x + r2.y) : 0.f;
        l2 = fmaf(r, r, l2);
      }
      lossacc += (double)l2;
    }
    const float wn = (float)(wold * (num * rden));  // SK:622-629 (div_nr's arithmetic)
    wt_[s * KK + e] = wn;
    if (!WRES) {  // lane l = (s, e); a resident tile's store goes to the dummy word
      if (!wr) reinterpret_cast<float*>(Wb)[(size_t)tile * TSW * KK + l] = wn;
      else asm volatile("global_store_dword %0, %1, off" ::"v"(dummy), "v"(0) : "memory");
    }
    // w'[s][·]: the sample's row back from LDS (this wave's writes above precede the reads)
    f2 wp[KP];
#pragma unroll
    for (int m4 = 0; m4 < KK / 4; ++m4) {
      const float4 v4 = *reinterpret_cast<const float4*>(wt_ + s * KK + 4 * m4);
      wp[2 * m4] = f2{v4.x, v4.y};
      wp[2 * m4 + 1] = f2{v4.z, v4.w};
    }
    // phase 3: A[·][f] += w'·x[f], B[e][·] += w'_e·w' (fp32 per lane over the iteration)
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      const f2 xx = f2{xv[c], xv[c]};
#pragma unroll
      for (int q = 0; q < KP; ++q) acc[c][q] = __builtin_elementwise_fma(xx, wp[q], acc[c][q]);
    }
#pragma unroll
    for (int q = 0; q < KP; ++q) accB[q] = __builtin_elementwise_fma(f2{wn, wn}, wp[q], accB[q]);
    if (i + 1 != nbt) return;

    // ---- end of this wave's iteration: its sums over the sample lanes of each e -> LDS
    // (reduce-scatter, round 6: value j = c·KK + 2q + comp (A), NQ·KK + 2q + comp (B); row r of the
    // wave ends with the quarter of the values scatter_over_samples names, written by the row's
    // lanes of sample 0, in pairs of floats)
    {
      float vv[NACC];
#pragma unroll
      for (int c = 0; c < NQ; ++c)
#pragma unroll
        for (int q = 0; q < KP; ++q) {
          vv[c * KK + 2 * q] = acc[c][q].x;
          vv[c * KK + 2 * q + 1] = acc[c][q].y;
        }
#pragma unroll
      for (int q = 0; q < KP; ++q) {
        vv[NQ * KK + 2 * q] = accB[q].x;
        vv[NQ * KK + 2 * q + 1] = accB[q].y;
      }
      scatter_over_samples<NL>(vv);
      constexpr int NQT = NACC / 4;
      static_assert(NQT % 2 == 0, "the quarters are written in pairs of floats");
      const int r = l >> 4;
      float* rw = red + (w * NL + e) * NACC + (NACC / 2) * (r >> 1) + NQT * (r & 1);
      if ((l & 15) < NL)
#pragma unroll
        for (int j = 0; j < NQT; j += 2) *reinterpret_cast<float2*>(rw + j) = make_float2(vv[j], vv[j + 1]);
    }
    zero_acc();
    if (TOL) {  // the wave's loss sum (zero outside loss iterations), fixed xor tree
      const double v = wave_sum(lossacc);
      if (l == 0) sLoss[w] = v;
      lossacc = 0.0;
    }
    __syncthreads();
    TL_PRE(it);
    // the workgroup's fp64 row [K][V] (+ the loss): the four waves' sums in wave order (deterministic)
    {
      double* prow = a.partials + (size_t)b * RS;
      const bool plain = sFlag[4] != 0;  // the group's rows through the XCD's L2 (l2rows)
      auto row_val = [&](int o) {
        const int j = o / V;
        const int v = o - j * V;
        const int ee = v < F ? v / NQ : j;
        const int idx = v < F ? (v - NQ * ee) * KK + j : NQ * KK + (v - F);
        const float* rr = red + ee * NACC + idx;
        constexpr int WS = NL * NACC;  // wave stride
        return ((double)rr[0] + (double)rr[WS]) + ((double)rr[2 * WS] + (double)rr[3 * WS]);
      };
      // pairs of doubles, one 16-byte store each (round 6); TOL: the loss at NOUT, a zero pad after it
      auto val = [&](int o) {
        if (o < NOUT) return row_val(o);
        return (TOL && o == NOUT) ? (sLoss[0] + sLoss[1]) + (sLoss[2] + sLoss[3]) : 0.0;
      };
      if constexpr (R6) {
        for (int c = t; c < RS / 2; c += NT) {
          const double v0 = val(2 * c), v1 = val(2 * c + 1);
          if (plain) st16_plain(prow + 2 * c, v0, v1);
          else st16_sc1v(prow + 2 * c, v0, v1);
        }
      } else {
        for (int o = t; o < NOUTT; o += NT) __hip_atomic_store(prow + o, val(o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores landed
    __syncthreads();
    TL(it, 0);
    if (t == 0) {
      const uint32_t old = __hip_atomic_fetch_add(cnt_group, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sFlag[0] = old == (uint32_t)((it + 1) * gs - 1);
      sFlag[1] = 0;
      sFlag[2] = 1;
      sFlag[3] = 0;
    }
    __syncthreads();
    // the last iteration of the launch waits for the flag too when it checks the tolerance (a stop
    // there must reach every workgroup before it writes W back)
    const bool must_wait = !last_it || loss_it;
    if (sFlag[0]) {  // group combiner
      TL_LV(it, g, 0);
      if constexpr (R6) sum_rows_v<RS>(a.partials, g, NG, gs, nullptr, a.groups + (size_t)g * RS, t);
      else sum_rows_n<RS>(a.partials, g, NG, gs, nullptr, a.groups + (size_t)g * RS, t);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      TL_LV(it, g, 1);
      if (t == 0) {
        const uint32_t old = __hip_atomic_fetch_add(cnt_top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sFlag[1] = old == (uint32_t)((it + 1) * NG - 1);
      }
      __syncthreads();
      if (sFlag[1]) {  // top combiner: AB
        TL_LV(it, TL_LVG, 0);
        if constexpr (R6) {
          sum_rows_v<RS>(a.groups, 0, 1, NG, sAB, a.AB, t);
          if (MULTI) __syncthreads();  // the exchange reads sAB in sum_rows_n's thread mapping
        } else {
          sum_rows_n<RS>(a.groups, 0, 1, NG, sAB, a.AB, t);
        }
        if (MULTI) xchg_allreduce_n<NOUTT>(a.xctl, a.AB, sAB, err, it, t);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        TL_LV(it, TL_LVG, 1);
        // (after the barrier: the summed loss sAB[NOUT] was written by another thread)
        if (TOL && loss_it && t == 0) {  // SK:872-884 on the state after it0 + it iterations
          const int gi = it0 + it;
          const double errv = sqrt(fmax(sAB[NOUT], 0.0));
          const int slot = gi / 10;
          if (slot < (int)ld_sc1(a.tolctl + TC_CAP)) st_sc1(a.tolctl + TC_ERRS + slot, errv);
          st_sc1(a.tolctl + TC_NERR, (double)(slot + 1));
          if (gi == 0) {
            sLoss[4] = sLoss[5] = errv;
            st_sc1(a.tolctl + TC_INIT, errv);
            st_sc1(a.tolctl + TC_PREV, errv);
          } else if ((sLoss[5] - errv) / sLoss[4] < tolv) {
            sFlag[3] = 1;
          } else {
            sLoss[5] = errv;
            st_sc1(a.tolctl + TC_PREV, errv);
          }
        }
        if (TOL && loss_it) __syncthreads();  // sFlag[3] (the decision) for the whole workgroup
        if (t == 0 && must_wait)
          __hip_atomic_store(flag, (uint32_t)(it + 1) | (sFlag[3] ? FLAG_STOP : 0u), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        TL_PUB(it);
      }
    }
    const bool top = sFlag[1] != 0;
    if (!top && must_wait) {
      if (t == 0) {
        const uint32_t want = (uint32_t)(it + 1);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t f;
        while (true) {  // the flag and the error word in one batch: one round trip per round
          const uint32_t ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((f & ~FLAG_STOP) >= want) break;
          if (ev != 0u) {
            sFlag[2] = 0;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > sl::SPIN_TIMEOUT) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sFlag[2] = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (TOL && (f & FLAG_STOP)) sFlag[3] = 1;
        TL_SEEN(it);
      }
      __syncthreads();
      if (!sFlag[2]) {  // a workgroup never arrived (not co-resident): give up, error word set
        alive = false;
        return;
      }
    }
    if (TOL && sFlag[3]) {
      // stopped by the tolerance test: the state after it0 + it iterations (W: the loss
      // iteration's LDS snapshot written back here, or the host copies the streamed-W snapshot
      // buffer; H = sH not updated); the host clears the flag word after the launch
      alive = false;
      if (WRES)
        for (int c = l; c < nbt * (WBW / 16); c += 64) {
          const int ii = c / (WBW / 16), ch = c - ii * (WBW / 16);
          *reinterpret_cast<u32x4*>(Wb + (size_t)(gw + (int64_t)NW * ii) * WBW + 16 * ch) =
              *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(wsnapl) + ii * WBW + 16 * ch);
        }
      if (!top) return;
      for (int o = t; o < KK * F; o += NT) a.H64[o] = sH[o];
      for (int o = t; o < F * KK; o += NT) {
        const int f = o / KK;
        const int j = o - f * KK;
        a.Ht[o] = sH[j * F + f];
      }
      if (t < KK * KK) a.HHt[t] = reinterpret_cast<const double*>(smem + G_::L_HHT)[t];
      if (t < NG) __hip_atomic_store(a.cnt + CNT_GROUP0 + 32 * t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (l2rows)
        for (int o = t; o < G; o += NT) __hip_atomic_store(a.cnt + CNT_XCC0 + o, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == 0) {
        __hip_atomic_store(cnt_top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st_sc1(a.tolctl + TC_DONE, (double)(it0 + it));
        st_sc1(a.tolctl + TC_STOPPED, 1.0);
        st_sc1(a.tolctl + TC_IN_SNAP, WRES ? 0.0 : 1.0);
        if (MULTI)
          __hip_atomic_fetch_add(a.xctl + XC_GEN, (uint64_t)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (last_it) {
      alive = false;
      if (WRES || nres > 0)  // this wave's resident W back to HBM, once per launch
        for (int c = l; c < (WRES ? nbt : min(nres, nbt)) * (WBW / 16); c += 64) {
          const int ii = c / (WBW / 16), ch = c - ii * (WBW / 16);
          *reinterpret_cast<u32x4*>(Wb + (size_t)(gw + (int64_t)NW * ii) * WBW + 16 * ch) =
              *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(wres) + ii * WBW + 16 * ch);
        }
      if (!top) return;
      // the last combiner of the launch: every other workgroup has arrived for the last time
      if (a.apply_last) {
        if constexpr (R6) wt_update_basis<KK>(smem, t, a.l1H, a.l2H);
        else wt_update_basis_r5<KK>(smem, t, a.l1H, a.l2H);
      }
      for (int o = t; o < KK * F; o += NT) a.H64[o] = sH[o];
      for (int o = t; o < F * KK; o += NT) {
        const int f = o / KK;
        const int j = o - f * KK;
        a.Ht[o] = sH[j * F + f];
      }
      if (t < KK * KK) a.HHt[t] = reinterpret_cast<const double*>(smem + G_::L_HHT)[t];
      if (t < NG) __hip_atomic_store(a.cnt + CNT_GROUP0 + 32 * t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (l2rows)
        for (int o = t; o < G; o += NT) __hip_atomic_store(a.cnt + CNT_XCC0 + o, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == 0) {
        __hip_atomic_store(cnt_top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!must_wait)  // (else workgroups may still poll it: the host clears it after the launch)
          __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (TOL) {
          st_sc1(a.tolctl + TC_DONE, (double)(it0 + a.n_iter));
          st_sc1(a.tolctl + TC_STOPPED, 0.0);
        }
        if (MULTI)  // the next launch's generations follow this one's
          __hip_atomic_fetch_add(a.xctl + XC_GEN, (uint64_t)a.n_iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (!top) {
      if constexpr (!R6) {
        for (int o = t; o < NOUTT; o += NT) sAB[o] = ld_sc1(a.AB + o);
      } else {  // 16-byte sc1 loads, all in flight together (round 6)
        constexpr int NCH = RS / 2;
        const int c0 = t < NCH ? t : 0, c1 = t + NT < NCH ? t + NT : 0;
        u32x4 r0, r1;
        ld16_sc1(r0, a.AB + 2 * c0);
        if (NCH > NT) ld16_sc1(r1, a.AB + 2 * c1);
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(r0), "+v"(r1) : : "memory");
        if (t < NCH) {
          sAB[2 * t] = lo_d(r0);
          sAB[2 * t + 1] = hi_d(r0);
        }
        if (t + NT < NCH) {
          sAB[2 * (t + NT)] = lo_d(r1);
          sAB[2 * (t + NT) + 1] = hi_d(r1);
        }
      }
      __syncthreads();
      TL_AB(it);
      if (TOL && loss_it && t == 0) {  // the top went on: prev <- this check's error
        const double errv = sqrt(fmax(sAB[NOUT], 0.0));
        if (it0 + it == 0) sLoss[4] = errv;
        sLoss[5] = errv;
      }
    }
    if (l2rows && it == 0 && w == 0) {
      // every member has written its XCC (at its start, before its first arrival): the group's rows
      // may go through the L2 when all of them share this workgroup's XCC (the same answer in every
      // member: they read the same table)
      const uint32_t xm = l < gs ? __hip_atomic_load(a.cnt + CNT_XCC0 + g + NG * l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : (uint32_t)sFlag[5];
      const bool same = __ballot(xm != (uint32_t)sFlag[5]) == 0;
      if (l == 0) sFlag[4] = same ? 1 : 0;
    }
    if constexpr (R6) wt_update_basis<KK>(smem, t, a.l1H, a.l2H);
    else wt_update_basis_r5<KK>(smem, t, a.l1H, a.l2H);
    TL_UPD(it);
    load_basis();
    TL(it, 1);
  };

  for (int p = 0; p < total && alive; p += PD) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      step(pf[k]);
      if (p + k < total && alive) body();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
}

// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// mu_iter_mf8_kernel<WRES, PD, MULTI, TOL> — k = 8 (cfg3) wave tiles on the matrix cores.
//
// The VALU wave-tile kernel at k = 8 is issue-bound (248 VALU per 8-sample tile against an FMA
// minimum of 85: the fp32 products plus the DPP reduce-scatter, fp64 folds and division; DESIGN
// §3.0).  Here both products run on v_mfma_f32_16x16x4_f32 (exact fp32 FMA chains at the f32
// rate), which issue beside the VALU work left (folds, the fp64 update, addressing), so the pass
// can become HBM-bound.  One wave owns 16-sample tiles (5184 B of X: the k = 4 tile geometry).
//   phase 1  NUM[s][e] = Σ_f x[s][f]·H[e][f]     M = 16 samples, N = 16 (8 components), K = 84:
//            21 K-steps in 7 independent chains of 3 (12 features each, ≤ the 14-rounding depth of
//            the VALU path), each chain folded into fp64 (DESIGN §4's long-fp32-dot hazard).
//            A = X[s = l&15][f = 4ks + l>>4] (LDS), B = Hᵀ[f][e = l&15] (21 VGPRs per basis).
//   phase 2  DEN[s][e] = Σ_m w[s][m]·HHᵀ[m][e]    2 MFMAs (fp32, 8 terms as the VALU path); the
//            update w·num/den in fp64 by the lanes e < 8 (4 samples each, the C layout
//            col = e = l&15, row = s = 4(l>>4) + r), SK:553-629.
//   phase 3  Aᵀ[f][n] = Σ_s [X | W'][s][f]·W'[s][n]   M = 16 features × 6 blocks (96 ≥ F + 8: the
//            last block's rows 81..88 carry W', so it also yields WᵀW), N = 16 (8 components),
//            K = 16 samples: 24 MFMAs in 6 independent accumulators, folded into fp64 every 16
//            tiles (≤ 256 samples per fp32 chain).
// W' reaches phase 3 through a [16][16] per-wave LDS image (columns ≥ 8 zero).  The prefetch /
// staging (AGPR sets, counted waits), the W residency, the end-of-iteration reduction, the
// in-launch exchange (MULTI) and the device tolerance test (TOL: ‖x − w·H‖² via 12 more MFMAs
// R = W·H in the loss iterations) are mu_iter_wt_kernel's.
// ------------------------------------------------------------------------------------------------
namespace wt {
typedef float f4v __attribute__((ext_vector_type(4)));
struct GeoMF8 {
  static constexpr int K = 8, TSW = 16, V = F + 8, NOUT = 8 * V;
  static constexpr int NL = 8, NQ = 11;  // the sHt image wt_derive_basis<8> writes (Geo<8>'s)
  static constexpr int XBW = TSW * F * 4;                  // 5184 B of X per tile
  static constexpr int NCHW = XBW / 16;                    // 324 chunks
  static constexpr int PFW = (NCHW + 63) / 64;             // 6 loads per lane
  static constexpr int LASTL = NCHW - 64 * (PFW - 1);      // 4
  static constexpr int PADB = 16;                          // phase 1 reads 3 floats past the tile
  static constexpr int XSTR = XBW + PADB;
  static constexpr int WBW = TSW * 8 * 4;                  // 512 B of W per tile
  static constexpr int KS1 = 21, NCH1 = 7, NB3 = 6;
  static constexpr int L_STG = 0;                                       // [NWV][XSTR]
  static constexpr int L_WSTG = L_STG + NWV * XSTR;                     // streamed W: [NWV][WBW]
  static constexpr int L_WP = (L_WSTG + NWV * WBW + 15) / 16 * 16;      // W' operand [NWV][16][16] fp32
  static constexpr int L_RED = L_WP + NWV * 16 * 16 * 4;                // [NWV][8][V] fp64
  static constexpr int L_H = L_RED + NWV * 8 * V * 8;                   // H fp64 [8][F]
  static constexpr int L_AB = L_H + 8 * F * 8;                          // AB fp64 (+ the loss)
  static constexpr int L_HT = L_AB + (NOUT + 2) * 8;                    // (wt_derive_basis' Hᵀ image)
  static constexpr int L_HHT = L_HT + NL * NQ * 8 * 4;                  // HHᵀ fp64 [8][8]
  static constexpr int L_FLAG = L_HHT + 8 * 8 * 8;                      // 8 ints
  static constexpr int L_LOSS = L_FLAG + 32;                            // [NWV] wave loss sums, init, prev
  static constexpr int L_WRES = (L_LOSS + 8 * 8 + 15) / 16 * 16;        // [NWV][nbt_max][WBW]
  static_assert(NCHW * 16 == XBW && L_HT % 16 == 0 && L_RED % 16 == 0, "layout");
  static_assert(NOUT * 8 >= NWV * 64 * 4, "the prologue's dummy stores stay inside the partial row");
};
__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
}  // namespace wt

template <bool WRES, int PD, bool MULTI = false, bool TOL = false>
__global__ __launch_bounds__(NT, 1) void mu_iter_mf8_kernel(PersistArgs a) {
  using namespace wt;
  using G_ = GeoMF8;
  constexpr int KK = 8, TSW = G_::TSW, V = G_::V, NOUT = G_::NOUT;
  constexpr int NOUTT = NOUT + (TOL ? 1 : 0);
  constexpr int XBW = G_::XBW, XSTR = G_::XSTR, WBW = G_::WBW, PFW = G_::PFW, LASTL = G_::LASTL;
  constexpr int PFS = PFW + (WRES ? 0 : 1);
  constexpr int NSTB = (WRES ? 0 : 1) + (TOL ? 1 : 0);  // stores per body (W streamed; TOL's snapshot)
  constexpr int KS1 = G_::KS1, NCH1 = G_::NCH1, NB3 = G_::NB3;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int t = threadIdx.x;
  const int l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lc = l & 15, lr = l >> 4;  // MFMA lane coordinates: column / row-group
  const int b = blockIdx.x;
  const int G = gridDim.x;
  const int NW = NWV * G;
  const int gw = NWV * b + w;
  const int NG = a.n_groups;
  const int g = b % NG;
  const int gs = (G - g + NG - 1) / NG;
  const unsigned char* Xb = reinterpret_cast<const unsigned char*>(a.X);
  unsigned char* Wb = reinterpret_cast<unsigned char*>(a.W);
  const int nbt = (int)((a.n_tiles - gw + NW - 1) / NW);
  const int nbt_max = (int)((a.n_tiles + NW - 1) / NW);
  unsigned char* stg = smem + G_::L_STG + w * XSTR;
  unsigned char* wstg = smem + G_::L_WSTG + w * WBW;
  float* wp = reinterpret_cast<float*>(smem + G_::L_WP) + w * 256;  // W' [16][16]
  float* wres = reinterpret_cast<float*>(smem + G_::L_WRES + (size_t)w * nbt_max * WBW);
  double* red = reinterpret_cast<double*>(smem + G_::L_RED);
  double* sH = reinterpret_cast<double*>(smem + G_::L_H);
  double* sAB = reinterpret_cast<double*>(smem + G_::L_AB);
  int* sFlag = reinterpret_cast<int*>(smem + G_::L_FLAG);
  double* sLoss = reinterpret_cast<double*>(smem + G_::L_LOSS);
  const int it0 = TOL ? (int)ld_sc1(a.tolctl + TC_IT0) : 0;
  // TOL: every workgroup tracks the test's error at init and previous error itself (sLoss[4], [5]),
  // so the decision of the iteration's top combiner reads no state another workgroup wrote
  const double tolv = TOL ? ld_sc1(a.tolctl + TC_TOL) : 0.0;
  if (TOL && t == 0) {
    sLoss[4] = ld_sc1(a.tolctl + TC_INIT);
    sLoss[5] = ld_sc1(a.tolctl + TC_PREV);
  }
  float* wsnap = (TOL && !WRES)
                     ? reinterpret_cast<float*>(__double_as_longlong(ld_sc1(a.tolctl + TC_WSNAP)))
                     : nullptr;
  double lossacc = 0.0;
  uint32_t* cnt_group = a.cnt + CNT_GROUP0 + 32 * g;
  uint32_t* cnt_top = a.cnt + CNT_TOP;
  uint32_t* flag = a.cnt + CNT_FLAG;
  uint32_t* err = a.cnt + CNT_ERR;

  for (int i = t; i < KK * F; i += NT) sH[i] = a.H64[i];
  if (a.apply_first)
    for (int i = t; i < NOUT; i += NT) sAB[i] = a.AB[i];
  if (l < G_::PADB / 4) reinterpret_cast<float*>(stg + XBW)[l] = 0.f;
  for (int i = l; i < 256; i += 64) wp[i] = 0.f;  // columns >= 8 stay zero for the launch
  if (WRES)
    for (int c = l; c < nbt * (WBW / 16); c += 64) {
      const int i = c / (WBW / 16), ch = c - i * (WBW / 16);
      *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned char*>(wres) + i * WBW + 16 * ch) =
          *reinterpret_cast<const u32x4*>(Wb + (size_t)(gw + (int64_t)NW * i) * WBW + 16 * ch);
    }
  __syncthreads();
  if (a.apply_first)
    wt_update_basis<KK, G_>(smem, t, a.l1H, a.l2H);
  else
    wt_derive_basis<KK, G_>(smem, t);

  // MFMA operands of the basis: Hᵀ[f = 4ks + lr][e = lc] (phase 1), HHᵀ[m = 4ks + lr][e = lc]
  // (DEN), H[m = 4ks + lr][f = 16 blk + lc] (TOL: R = W·H); zero past k = 8 / F
  float hB[KS1], hhB[2], hR[TOL ? NB3 : 1][2];
  auto load_basis = [&]() {
    const double* sHHt = reinterpret_cast<const double*>(smem + G_::L_HHT);
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      const int f = 4 * ks + lr;
      hB[ks] = (lc < KK && f < F) ? (float)sH[(lc & 7) * F + (f < F ? f : 0)] : 0.f;
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) hhB[ks] = lc < KK ? (float)sHHt[(4 * ks + lr) * KK + (lc & 7)] : 0.f;
    if constexpr (TOL)
#pragma unroll
      for (int blk = 0; blk < NB3; ++blk)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int f = 16 * blk + lc;
          hR[blk][ks] = f < F ? (float)sH[(4 * ks + lr) * F + (f < F ? f : 0)] : 0.f;
        }
  };
  load_basis();

  // phase-3 accumulators: fp32 MFMA C (≤ 16 tiles), fp64 folds; lane holds Aᵀ[16 blk + 4 lr + r][lc]
  f4v acc3[NB3];
  double acc64[NB3][4];
  auto zero32 = [&]() {
#pragma unroll
    for (int blk = 0; blk < NB3; ++blk) acc3[blk] = f4v{0.f, 0.f, 0.f, 0.f};
  };
  auto fold = [&]() {
#pragma unroll
    for (int blk = 0; blk < NB3; ++blk)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc64[blk][r] += (double)acc3[blk][r];
    zero32();
  };
  zero32();
#pragma unroll
  for (int blk = 0; blk < NB3; ++blk)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc64[blk][r] = 0.0;

  auto prefetch = [&](u32x4 (&pf)[PFS], int64_t tile) {
    const unsigned char* xs = Xb + (size_t)tile * XBW + 16 * l;
#pragma unroll
    for (int u = 0; u < PFW - 1; ++u) ld16(pf[u], xs + 1024 * u);
    ld16(pf[PFW - 1], l < LASTL ? xs + 1024 * (PFW - 1) : xs);
    if (!WRES) ld16(pf[PFW], l < WBW / 16 ? Wb + (size_t)tile * WBW + 16 * l : xs);
  };
  auto stage = [&](const u32x4 (&pf)[PFS]) {
    const unsigned addr = (unsigned)(uintptr_t)(stg + 16 * l);
    stage_rec<0, PFW - 1>(addr, pf);
    if (l < LASTL) st16<1024 * (PFW - 1)>(addr, pf[PFW - 1]);
    if (!WRES && l < WBW / 16) st16<0>((unsigned)(uintptr_t)(wstg + 16 * l), pf[PFW]);
  };

  const int total = a.n_iter * nbt;
  u32x4 pf[PD][PFS];
  float* dummy = reinterpret_cast<float*>(a.partials + (size_t)b * NOUTT) + 64 * w + l;
#pragma unroll
  for (int k = 0; k < PD; ++k) {
    prefetch(pf[k], gw + (int64_t)NW * k);
#pragma unroll
    for (int d = 0; d < NSTB; ++d) asm volatile("global_store_dword %0, %1, off" ::"v"(dummy), "v"(0) : "memory");
  }
  TL_START;

  bool alive = true;
  int cur_i = 0, cur_it = 0, nx_i = PD;
  auto step = [&](u32x4 (&pfk)[PFS]) {
    wait_set<PFS * (PD - 1) + NSTB * PD, PFS>(pfk);  // (the stores per body: mu_iter_wt_kernel's step)
    stage(pfk);
    prefetch(pfk, gw + (int64_t)NW * nx_i);
    if (++nx_i == nbt) nx_i = 0;
  };
  auto body = [&]() {
    const int it = cur_it, i = cur_i;
    if (++cur_i == nbt) {
      cur_i = 0;
      ++cur_it;
    }
    const bool last_it = it + 1 == a.n_iter;
    const bool loss_it = TOL && ((it0 + it) % 10 == 0);
    const int64_t tile = gw + (int64_t)NW * i;
    const float* sx = reinterpret_cast<const float*>(stg);
    float* wt_ = WRES ? wres + i * (TSW * KK) : reinterpret_cast<float*>(wstg);  // [16][8]
    // ---- phase 1: NUM = X·Hᵀ on the matrix cores, 7 chains of 3 K-steps folded into fp64
    f4v c1[NCH1];
#pragma unroll
    for (int c = 0; c < NCH1; ++c) c1[c] = f4v{0.f, 0.f, 0.f, 0.f};
    {
      const float* xa = sx + lc * F + lr;  // A = X[s = lc][f = 4 ks + lr]
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int c = 0; c < NCH1; ++c) {
          const int ks = 3 * c + j;
          c1[c] = mfma4(xa[4 * ks], hB[ks], c1[c]);
        }
    }
    // ---- DEN = W·HHᵀ (A = W[s = lc][m = 4 ks + lr])
    const float wa0 = wt_[lc * KK + lr], wa1 = wt_[lc * KK + 4 + lr];
    f4v dn = mfma4(wa0, hhB[0], f4v{0.f, 0.f, 0.f, 0.f});
    dn = mfma4(wa1, hhB[1], dn);
    if (loss_it) {
      // ‖x − w·H‖² of the state before this update: R = W·H (C[s = 4 lr + r][f = 16 blk + lc])
      float l2 = 0.f;
#pragma unroll
      for (int blk = 0; blk < NB3; ++blk) {
        f4v rr = mfma4(wa0, hR[blk][0], f4v{0.f, 0.f, 0.f, 0.f});
        rr = mfma4(wa1, hR[blk][1], rr);
        const int f = 16 * blk + lc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = sx[(4 * lr + r) * F + (f < F ? f : 0)];
          const float d = f < F ? x - rr[r] : 0.f;
          l2 = fmaf(d, d, l2);
        }
      }
      lossacc += (double)l2;
    }
    if constexpr (TOL) {
      // the W of the checked state (16 B per lane of the first 32), ONE store per body in every
      // iteration (counted by the steps' waits): a loss iteration's into W itself (resident W) or
      // the snapshot buffer (streamed W), the others' over the wave's first tile there (overwritten
      // by the next loss iteration or the launch's write-back; mu_iter_wt_kernel's snapshot)
      if (l < WBW / 16) {
        const u32x4 wv16 = *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(wt_) + 16 * l);
        unsigned char* dst = WRES ? Wb : reinterpret_cast<unsigned char*>(wsnap);
        const int64_t tsel = loss_it ? tile : (int64_t)gw;
        *reinterpret_cast<u32x4*>(dst + (size_t)tsel * WBW + 16 * l) = wv16;
      }
    }
    // ---- phase 2: the update of (s = 4 lr + r, e = lc) for e < 8, fp64 (SK:553-629)
    {
      const int e = lc & 7;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int s = 4 * lr + r;
        const double num = ((((double)c1[0][r] + (double)c1[1][r]) + ((double)c1[2][r] + (double)c1[3][r])) +
                            (((double)c1[4][r] + (double)c1[5][r]) + (double)c1[6][r]));
        const double wold = (double)wt_[s * KK + e];
        double den = (double)dn[r];
        if (a.l1W > 0.0) den += a.l1W;              // SK:616-617
        if (a.l2W > 0.0) den = den + a.l2W * wold;  // SK:618-619
        if (den == 0.0) den = EPS32;                // SK:620
        const float wn = (float)(wold * div_nr(num, den));  // SK:622-629
        if (lc < KK) {
          wt_[s * KK + e] = wn;
          wp[s * 16 + e] = wn;
        }
      }
    }
    if (!WRES) {  // the tile's new W to HBM: ONE 16-byte store instruction per body (the counted
                  // waits), lanes 32..63 repeating lanes 0..31's identical writes
      const int lw = l & 31;
      *reinterpret_cast<u32x4*>(Wb + (size_t)tile * WBW + 16 * lw) =
          *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(wt_) + 16 * lw);
    }
    // ---- phase 3: Aᵀ += [X | W']ᵀ·W' (B = W'[s = 4 ks + lr][n = lc]; A = [X | W'][s][f = 16 blk + lc])
    {
      float bw[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) bw[ks] = wp[(4 * ks + lr) * 16 + lc];
      const float* xb = sx + lr * F + lc;  // X[s = 4 ks + lr][f = 16 blk + lc]
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int blk = 0; blk < NB3; ++blk) {
          float av;
          if (blk < NB3 - 1) {
            av = xb[4 * ks * F + 16 * blk];
          } else {  // features 80..95: x[s][80], then W'[s][0..7] (-> WᵀW), then zero
            const float xv = xb[4 * ks * F + 16 * blk - lc];  // x[s][80] (clamped address)
            const float wv = wp[(4 * ks + lr) * 16 + ((lc - 1) & 7)];
            av = lc == 0 ? xv : (lc <= KK ? wv : 0.f);
          }
          acc3[blk] = mfma4(av, bw[ks], acc3[blk]);
        }
    }
    if ((i & 15) == 15) fold();  // ≤ 256 samples per fp32 chain
    if (i + 1 != nbt) return;

    // ---- end of this wave's iteration: its sums -> LDS [w][n][f] (fp64)
    fold();
    if (lc < KK)
#pragma unroll
      for (int blk = 0; blk < NB3; ++blk)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 16 * blk + 4 * lr + r;
          if (f < V) red[(w * KK + lc) * V + f] = acc64[blk][r];
        }
#pragma unroll
    for (int blk = 0; blk < NB3; ++blk)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc64[blk][r] = 0.0;
    if (TOL) {
      const double v = wave_sum(lossacc);
      if (l == 0) sLoss[w] = v;
      lossacc = 0.0;
    }
    __syncthreads();
    {
      double* prow = a.partials + (size_t)b * NOUTT;
      if (TOL && t == 0)
        __hip_atomic_store(prow + NOUT, (sLoss[0] + sLoss[1]) + (sLoss[2] + sLoss[3]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      for (int o = t; o < NOUT; o += NT) {
        constexpr int WS = KK * V;  // wave stride
        const double val = (red[o] + red[o + WS]) + (red[o + 2 * WS] + red[o + 3 * WS]);
        __hip_atomic_store(prow + o, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores landed
    __syncthreads();
    TL(it, 0);
    if (t == 0) {
      const uint32_t old = __hip_atomic_fetch_add(cnt_group, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sFlag[0] = old == (uint32_t)((it + 1) * gs - 1);
      sFlag[1] = 0;
      sFlag[2] = 1;
      sFlag[3] = 0;
    }
    __syncthreads();
    // the last iteration of the launch waits for the flag too when it checks the tolerance (a stop
    // there must reach every workgroup before it writes W back)
    const bool must_wait = !last_it || loss_it;
    if (sFlag[0]) {  // group combiner
      sum_rows_n<NOUTT>(a.partials, g, NG, gs, nullptr, a.groups + (size_t)g * NOUTT, t);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) {
        const uint32_t old = __hip_atomic_fetch_add(cnt_top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sFlag[1] = old == (uint32_t)((it + 1) * NG - 1);
      }
      __syncthreads();
      if (sFlag[1]) {  // top combiner: AB
        sum_rows_n<NOUTT>(a.groups, 0, 1, NG, sAB, a.AB, t);
        if (MULTI) xchg_allreduce_n<NOUTT>(a.xctl, a.AB, sAB, err, it, t);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // (after the barrier: the summed loss sAB[NOUT] was written by another thread)
        if (TOL && loss_it && t == 0) {  // SK:872-884 on the state after it0 + it iterations
          const int gi = it0 + it;
          const double errv = sqrt(fmax(sAB[NOUT], 0.0));
          const int slot = gi / 10;
          if (slot < (int)ld_sc1(a.tolctl + TC_CAP)) st_sc1(a.tolctl + TC_ERRS + slot, errv);
          st_sc1(a.tolctl + TC_NERR, (double)(slot + 1));
          if (gi == 0) {
            sLoss[4] = sLoss[5] = errv;
            st_sc1(a.tolctl + TC_INIT, errv);
            st_sc1(a.tolctl + TC_PREV, errv);
          } else if ((sLoss[5] - errv) / sLoss[4] < tolv) {
            sFlag[3] = 1;
          } else {
            sLoss[5] = errv;
            st_sc1(a.tolctl + TC_PREV, errv);
          }
        }
        if (TOL && loss_it) __syncthreads();  // sFlag[3] (the decision) for the whole workgroup
        if (t == 0 && must_wait)
          __hip_atomic_store(flag, (uint32_t)(it + 1) | (sFlag[3] ? FLAG_STOP : 0u), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        TL_PUB(it);
      }
    }
    const bool top = sFlag[1] != 0;
    if (!top && must_wait) {
      if (t == 0) {
        const uint32_t want = (uint32_t)(it + 1);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t f;
        while (true) {  // the flag and the error word in one batch: one round trip per round
          const uint32_t ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((f & ~FLAG_STOP) >= want) break;
          if (ev != 0u) {
            sFlag[2] = 0;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > sl::SPIN_TIMEOUT) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sFlag[2] = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (TOL && (f & FLAG_STOP)) sFlag[3] = 1;
      }
      __syncthreads();
      if (!sFlag[2]) {  // a workgroup never arrived (not co-resident): give up, error word set
        alive = false;
        return;
      }
    }
    if (TOL && sFlag[3]) {
      // stopped by the tolerance test: the state after it0 + it iterations (W already where it
      // belongs, H = sH not updated); the host clears the flag word after the launch
      alive = false;
      if (!top) return;
      for (int o = t; o < KK * F; o += NT) a.H64[o] = sH[o];
      for (int o = t; o < F * KK; o += NT) {
        const int f = o / KK;
        const int j = o - f * KK;
        a.Ht[o] = sH[j * F + f];
      }
      if (t < KK * KK) a.HHt[t] = reinterpret_cast<const double*>(smem + G_::L_HHT)[t];
      if (t < NG) __hip_atomic_store(a.cnt + CNT_GROUP0 + 32 * t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == 0) {
        __hip_atomic_store(cnt_top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st_sc1(a.tolctl + TC_DONE, (double)(it0 + it));
        st_sc1(a.tolctl + TC_STOPPED, 1.0);
        st_sc1(a.tolctl + TC_IN_SNAP, WRES ? 0.0 : 1.0);
        if (MULTI)
          __hip_atomic_fetch_add(a.xctl + XC_GEN, (uint64_t)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (last_it) {
      alive = false;
      if (WRES)  // this wave's W back to HBM, once per launch
        for (int c = l; c < nbt * (WBW / 16); c += 64) {
          const int ii = c / (WBW / 16), ch = c - ii * (WBW / 16);
          *reinterpret_cast<u32x4*>(Wb + (size_t)(gw + (int64_t)NW * ii) * WBW + 16 * ch) =
              *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(wres) + ii * WBW + 16 * ch);
        }
      if (!top) return;
      // the last combiner of the launch: every other workgroup has arrived for the last time
      if (a.apply_last) wt_update_basis<KK, G_>(smem, t, a.l1H, a.l2H);
      for (int o = t; o < KK * F; o += NT) a.H64[o] = sH[o];
      for (int o = t; o < F * KK; o += NT) {
        const int f = o / KK;
        const int j = o - f * KK;
        a.Ht[o] = sH[j * F + f];
      }
      if (t < KK * KK) a.HHt[t] = reinterpret_cast<const double*>(smem + G_::L_HHT)[t];
      if (t < NG) __hip_atomic_store(a.cnt + CNT_GROUP0 + 32 * t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == 0) {
        __hip_atomic_store(cnt_top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!must_wait)  // (else workgroups may still poll it: the host clears it after the launch)
          __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (TOL) {
          st_sc1(a.tolctl + TC_DONE, (double)(it0 + a.n_iter));
          st_sc1(a.tolctl + TC_STOPPED, 0.0);
        }
        if (MULTI)  // the next launch's generations follow this one's
          __hip_atomic_fetch_add(a.xctl + XC_GEN, (uint64_t)a.n_iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (!top) {
      for (int o = t; o < NOUTT; o += NT) sAB[o] = ld_sc1(a.AB + o);
      __syncthreads();
      if (TOL && loss_it && t == 0) {  // the top went on: prev <- this check's error
        const double errv = sqrt(fmax(sAB[NOUT], 0.0));
        if (it0 + it == 0) sLoss[4] = errv;
        sLoss[5] = errv;
      }
    }
    wt_update_basis<KK, G_>(smem, t, a.l1H, a.l2H);
    load_basis();
    TL(it, 1);
  };

  for (int p = 0; p < total && alive; p += PD) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      step(pf[k]);
      if (p + k < total && alive) body();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
}

// ------------------------------------------------------------------------------------------------
// Normalisation projection (build spec, no sklearn counterpart): every basis row
// H_j is rescaled to unit norm and the scale folded into column j of W, so W·H is unchanged:
//   s_j = ‖H_j‖ (norm 1: L1, 2: L2, 3: max), H_j <- H_j / s_j, W[:, j] <- W[:, j]·s_j
// (rows with s_j == 0 are left alone, s_j := 1).  One workgroup computes s (fp64, fixed-order wave
// sums), rewrites H64 and derives Ht / HHt; then a grid-stride pass scales W.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(RED_NT) void normalise_basis_kernel(double* __restrict__ H64,
                                                                 double* __restrict__ Ht,
                                                                 double* __restrict__ HHt,
                                                                 double* __restrict__ scale, int F,
                                                                 int k, int KP, int norm) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* ss = reinterpret_cast<double*>(smem);  // [16] scales
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  for (int j = wave; j < k; j += RED_NT / 64) {
    double v = 0.0;
    for (int f = lane; f < F; f += 64) {
      const double h = H64[j * F + f];
      if (norm == 1) v += fabs(h);
      else if (norm == 2) v = fma(h, h, v);
      else v = fmax(v, fabs(h));
    }
    if (norm == 3) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    } else {
      v = wave_sum(v);
    }
    if (norm == 2) v = sqrt(v);
    if (lane == 0) ss[j] = v > 0.0 ? v : 1.0;
  }
  __syncthreads();
  if (t < k) scale[t] = ss[t];
  for (int e = t; e < k * F; e += RED_NT) H64[e] = H64[e] / ss[e / F];
  __syncthreads();  // workgroup-scope fence + barrier: the H64 stores are visible to this workgroup
  basis_update_block(nullptr, H64, Ht, HHt, F, k, KP, 0.0, 0.0, 0, nullptr,
                     reinterpret_cast<double*>(smem) + 16);
}

template <typename TC>
__global__ __launch_bounds__(256) void scale_columns_kernel(TC* __restrict__ W, const double* __restrict__ scale,
                                                            int64_t n, int k) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += stride)
    W[e] = (TC)((double)W[e] * scale[e % k]);
}

// ------------------------------------------------------------------------------------------------
// Constrained ALS, basis side (the spec and its scipy-NNLS oracle:
// oracle/als_ref.py).  One workgroup, all fp64:
//   * H-step (do_update): one Gauss-Seidel sweep over the basis rows j = 0..k-1, each the exact
//     NNLS  h_j = argmin_{h>=0} ½hᵀ(B_jj I + λL)h - (a_j - Σ_{m≠j} B_jm h_m)ᵀh,  L = DᵀD (second
//     difference, pentadiagonal), by block principal pivoting (Kim & Park's BPP: swap every
//     infeasible index, fall back to single swaps when the infeasible count stops falling), warm
//     started from the row's current support.  The passive subsystem of a pentadiagonal matrix is
//     pentadiagonal in the compressed index order, so each solve is an O(F) banded Cholesky
//     (thread 0); the residuals and infeasibility tests run over all threads.
//   * Ht / HHt from the new H (basis_update_block), then the W-step's passive-set table for
//     Q = HHᵀ + δ²11ᵀ: per mask P (k <= 4) the inverse of Q_PP by Gauss-Jordan with partial
//     pivoting, scattered to 4x4 (zeros outside P), and a valid flag (pivot > 1e-13·max diag).
// ------------------------------------------------------------------------------------------------
constexpr int ALS_MAX_F = 512;
// components of the constrained ALS: the W-step's passive-set table (16 masks), the one-wave H-step's
// running right-hand-side update and its sweep-count slots are sized for it; every ALS entry point
// refuses k > ALS_MAX_K with CNMF_ERR_UNSUPPORTED before any launch
constexpr int ALS_MAX_K = 4;

__host__ __device__ inline size_t als_pre_offset(int F, int k) {  // 16-B aligned, after the ints
  return (((size_t)2 * k * F + k * k + 9 * (size_t)F) * 8 + (3 * (size_t)F + 16) * 4 + 15) / 16 * 16;
}
__host__ __device__ inline size_t als_lds_bytes(int F, int k) {
  // doubles: A, H [k][F]; B [k][k]; b, x, d0, e1, e2, L0, L1, L2, z [F]; then ints: pas, inf, idx [F], 8;
  // then (the one-wave form's per-row constants, round 5) bpre, rinv [k][F] and ALS_MAX_K sweep counts
  return als_pre_offset(F, k) + ((size_t)2 * k * F + ALS_MAX_K) * 8;
}

// M(fa, fb) of the row Hessian for |fa - fb| <= 2 (0 otherwise), fb < fa
__device__ __forceinline__ double als_m_low(const double* e1, const double* e2, int fa, int fb) {
  const int d = fa - fb;
  return d == 1 ? e1[fb] : (d == 2 ? e2[fb] : 0.0);
}

__device__ double als_L_entry(int F, int a, int b) {  // (DᵀD)[a][b], b >= a, |b - a| <= 2
  double v = 0.0;
  for (int r = a - 2; r <= a; ++r) {
    if (r < 0 || r > F - 3) continue;
    const int ia = a - r, ib = b - r;
    if (ib < 0 || ib > 2) continue;
    const double ca = ia == 1 ? -2.0 : 1.0;
    const double cb = ib == 1 ? -2.0 : 1.0;
    v += ca * cb;
  }
  return v;
}

// The H-step sweep in LDS (als_lds_bytes(F, k) bytes at smem, RED_NT threads): on entry sA [k][F] =
// WᵀX, sH [k][F] = the basis, sB [k][k] = WᵀW (the first three arrays of the layout); on return
// sH holds the new basis.  Deterministic: every workgroup that runs it on the same inputs gets the
// same bits (the LDS atomics only count and take a maximum).
#ifdef CNMF_STAMPS
// diagnostic: per H-step call of workgroup 0 (the first 64 calls) and row: BPP iterations, cycles
__device__ unsigned long long g_hs[64 * 4 * 2];
__device__ unsigned long long g_hsp[64 * 4 * 4];  // wave H-step: [call][row][setup, gather, PCR, check] cycles
__device__ unsigned int g_hs_calls;
#endif
__device__ __forceinline__ void als_hstep_block(unsigned char* smem, int F, int k, double lam, int t) {
#ifdef CNMF_STAMPS
  const unsigned hs_call = blockIdx.x == 0 ? __hip_atomic_load(&g_hs_calls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 64u;
#endif
  double* sA = reinterpret_cast<double*>(smem);
  double* sH = sA + (size_t)k * F;
  double* sB = sH + (size_t)k * F;
  double* vb = sB + k * k;
  double* vx = vb + F;
  double* d0 = vx + F;
  double* e1 = d0 + F;
  double* e2 = e1 + F;
  double* L0 = e2 + F;
  double* L1 = L0 + F;
  double* L2 = L1 + F;
  double* vz = L2 + F;
  int* pas = reinterpret_cast<int*>(vz + F);
  int* inf = pas + F;
  int* idx = inf + F;
  int* ctl = idx + F;  // [0] n_inf, [1] max infeasible index, [2] mode, [3] n passive
  {
    for (int j = 0; j < k; ++j) {
      const double bjj = sB[j * k + j];
      if (!(bjj > 0.0)) continue;  // unused component: row unchanged (oracle: same)
#ifdef CNMF_STAMPS
      const unsigned long long hs_t0 = __builtin_amdgcn_s_memtime();
      int hs_iters = 0;
#endif
      for (int f = t; f < F; f += RED_NT) {
        double b = sA[j * F + f];
        for (int m = 0; m < k; ++m)
          if (m != j) b -= sB[j * k + m] * sH[m * F + f];
        vb[f] = b;
        d0[f] = bjj + lam * als_L_entry(F, f, f);
        e1[f] = f + 1 < F ? lam * als_L_entry(F, f, f + 1) : 0.0;
        e2[f] = f + 2 < F ? lam * als_L_entry(F, f, f + 2) : 0.0;
        pas[f] = sH[j * F + f] > 0.0;
      }
      __syncthreads();
      int alpha = 3, beta = F + 1;  // BPP control (thread 0's copy is the one that counts)
      const int lane = t & 63, wave = t >> 6;
      for (int iter = 0; iter < 5 * F + 10; ++iter) {
        // ---- compress the passive set in parallel (ballot prefix per wave, waves in order;
        // per-wave counts in ctl[4 + 4c + wave])
        int pos[2];
        bool pp[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int f = c * RED_NT + t;
          pp[c] = f < F && pas[f];
          const uint64_t bal = __ballot(pp[c]);
          pos[c] = __popcll(bal & ((1ull << lane) - 1ull));
          if (lane == 0) ctl[4 + c * 4 + wave] = __popcll(bal);
        }
        for (int f = t; f < F; f += RED_NT) vx[f] = 0.0;
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          int base = 0;
          for (int u = 0; u < c * 4 + wave; ++u) base += ctl[4 + u];
          if (pp[c]) idx[base + pos[c]] = c * RED_NT + t;
        }
        if (t == 0) {
          int nn = 0;
          for (int u = 0; u < 8; ++u) nn += ctl[4 + u];
          ctl[3] = nn;
        }
        __syncthreads();
        const int n = ctl[3];
        // compressed Hessian entries and right-hand side, in parallel
        for (int a = t; a < n; a += RED_NT) {
          const int fa = idx[a];
          L0[a] = d0[fa];                                            // M_aa
          L1[a] = a >= 1 ? als_m_low(e1, e2, fa, idx[a - 1]) : 0.0;  // M_a,a-1
          L2[a] = a >= 2 ? als_m_low(e1, e2, fa, idx[a - 2]) : 0.0;  // M_a,a-2
          vz[a] = vb[fa];
        }
        __syncthreads();
        if (t == 0) {
          // banded LDLᵀ (unit L, bandwidth 2) fused with the forward solve L z = b, then
          // x = L⁻ᵀ D⁻¹ z; the recurrences are carried in registers, one reciprocal per step.
          // Since l_{a,a-2}·d_{a-2} = m_{a,a-2}: u1 = m_{a,a-1} − m_{a,a-2}·l_{a-1,a-2} is the
          // unscaled l_{a,a-1}, and d_a = m_aa − l2·m_{a,a-2} − l1·u1, so the loop-carried cycle is
          // id_{a-1} -> l1 -> d -> id_a (7 dependent fp64 ops).  The next step's four LDS values are
          // loaded one step ahead (their latency hides behind that cycle).
          double im1 = 0.0, im2 = 0.0, l1m1 = 0.0, zm1 = 0.0, zm2 = 0.0;
          double n_aa = n > 0 ? L0[0] : 1.0, n_a1 = 0.0, n_a2 = 0.0, n_b = n > 0 ? vz[0] : 0.0;
          for (int a = 0; a < n; ++a) {
            const double m_aa = n_aa, m_a1 = n_a1, m_a2 = n_a2, b = n_b;
            if (a + 1 < n) {
              n_aa = L0[a + 1];
              n_a1 = L1[a + 1];
              n_a2 = L2[a + 1];
              n_b = vz[a + 1];
            }
            const double l2 = m_a2 * im2;                  // l_{a,a-2}
            const double u1 = fma(-m_a2, l1m1, m_a1);      // l_{a,a-1}·d_{a-1}
            const double l1 = u1 * im1;                    // l_{a,a-1}
            const double d = fmax(fma(-l1, u1, fma(-l2, m_a2, m_aa)), 1e-300);
            // 1/d: v_rcp_f64 refined by two Newton steps (full fp64 accuracy)
            double id = __builtin_amdgcn_rcp(d);
            id = fma(id, fma(-d, id, 1.0), id);
            id = fma(id, fma(-d, id, 1.0), id);
            const double z = fma(-l2, zm2, fma(-l1, zm1, b));
            L1[a] = l1;
            L2[a] = l2;
            vz[a] = z * id;  // y = D⁻¹ z
            im2 = im1; im1 = id; l1m1 = l1; zm2 = zm1; zm1 = z;
          }
          double xp1 = 0.0, xp2 = 0.0, l1p1 = 0.0, l2p1 = 0.0, l2p2 = 0.0;
          double n_y = n > 0 ? vz[n - 1] : 0.0, n_l1 = n > 0 ? L1[n - 1] : 0.0, n_l2 = n > 0 ? L2[n - 1] : 0.0;
          for (int a = n - 1; a >= 0; --a) {
            const double y = n_y, la1 = n_l1, la2 = n_l2;
            if (a > 0) {
              n_y = vz[a - 1];
              n_l1 = L1[a - 1];
              n_l2 = L2[a - 1];
            }
            // x_a = y_a - l_{a+1,a} x_{a+1} - l_{a+2,a} x_{a+2}
            const double x = fma(-l2p2, xp2, fma(-l1p1, xp1, y));
            vz[a] = x;
            xp2 = xp1; xp1 = x;
            l2p2 = l2p1; l2p1 = la2; l1p1 = la1;
          }
          ctl[0] = 0;
          ctl[1] = -1;
        }
        __syncthreads();
        for (int a = t; a < n; a += RED_NT) vx[idx[a]] = vz[a];
        __syncthreads();
        for (int f = t; f < F; f += RED_NT) {
          const double x = vx[f];
          bool bad;
          if (pas[f]) {
            bad = x < 0.0;
          } else {
            double y = d0[f] * x - vb[f];
            if (f + 1 < F) y += e1[f] * vx[f + 1];
            if (f >= 1) y += e1[f - 1] * vx[f - 1];
            if (f + 2 < F) y += e2[f] * vx[f + 2];
            if (f >= 2) y += e2[f - 2] * vx[f - 2];
            bad = y < 0.0;
          }
          inf[f] = bad;
          if (bad) {
            atomicAdd(&ctl[0], 1);
            atomicMax(&ctl[1], f);
          }
        }
        __syncthreads();
        if (t == 0) {
          const int ninf = ctl[0];
          int mode;
          if (ninf == 0) mode = 0;
          else if (ninf < beta) { beta = ninf; alpha = 3; mode = 1; }
          else if (alpha >= 1) { --alpha; mode = 1; }
          else mode = 2;
          ctl[2] = mode;
        }
        __syncthreads();
        const int mode = ctl[2];
#ifdef CNMF_STAMPS
        ++hs_iters;
#endif
        if (mode == 0) break;
        for (int f = t; f < F; f += RED_NT)
          if ((mode == 1 && inf[f]) || (mode == 2 && f == ctl[1])) pas[f] ^= 1;
        __syncthreads();
      }
      for (int f = t; f < F; f += RED_NT) sH[j * F + f] = fmax(vx[f], 0.0);
      __syncthreads();
#ifdef CNMF_STAMPS
      if (t == 0 && hs_call < 64u && j < 4) {
        g_hs[(hs_call * 4 + j) * 2] = (unsigned long long)hs_iters;
        g_hs[(hs_call * 4 + j) * 2 + 1] = __builtin_amdgcn_s_memtime() - hs_t0;
      }
#endif
    }
  }
#ifdef CNMF_STAMPS
  if (t == 0 && blockIdx.x == 0) __hip_atomic_fetch_add(&g_hs_calls, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }
// The value through an empty asm: what is derived from it can no longer be hoisted out of a
// persistent kernel's iteration loop.  (The compiler hoisted the end-of-iteration code's lane
// addresses — LDS row offsets, the butterflies' ds_bpermute addresses — and, short of registers
// across the streaming loop, spilled them: each reload in the reduction / H-step / derive path was
// a scratch round trip, behind a vmcnt(0) that also waited for the in-flight prefetch.)
__device__ __forceinline__ int opaque_i(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ double opaque_d(double v) {
  asm volatile("" : "+v"(v));
  return v;
}

// The same sweep for F <= 128 on ONE wave, without a workgroup barrier inside it (same LDS layout;
// the other waves wait at the closing barrier).  Lane l holds features 2l and 2l + 1 (round 5: the
// pair layout), so a feature's neighbours f ± 1, f ± 2 are the lane's other feature or one of the
// two adjacent lanes' pair: the Jacobi sweeps and the dual checks fetch them with wave_shr / wave_shl
// DPP moves (a few cycles) instead of an LDS store + read round trip per sweep.  (The rows of WᵀX
// and H are still read from LDS per row: holding all k rows in registers raised the persistent
// kernel's spills from 26 to 72 VGPRs, where the reads are one batch per row.)  Rows whose Jacobi
// contraction bound is not small take the block PCR: the passive set compressed by ballots and each
// solve M_PP x = b_P a parallel cyclic reduction over 2x2 blocks of the compressed pentadiagonal
// system (log2(n/2) steps of register arithmetic and lane shuffles) instead of the n sequential steps
// of a banded LDLᵀ, whose loop-carried chain of ~10 dependent fp64 operations made a row cost
// 20-40 k cycles (profiles/r02/session5/als_diag).  The arithmetic of every value — the same fused
// operations in the same order, neighbours outside the row entering with zero coefficients — is
// unchanged from the lane = (f, f + 64) form: the sweep's result is the same bits.
__device__ __forceinline__ double dpp_wave_shr(double v) {  // lane i <- lane i - 1 (lane 0: 0)
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_wave_shl(double v) {  // lane i <- lane i + 1 (lane 63: 0)
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x130, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void als_hstep_wave(unsigned char* smem, int F, int k, double lam, int t) {
#ifdef CNMF_STAMPS
  const unsigned hs_call = blockIdx.x == 0 ? __hip_atomic_load(&g_hs_calls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 64u;
#endif
  // ---- round 5: what every row needs from the OLD basis and from B alone, by all the workgroup's
  // threads in parallel before the sequential sweep (the one wave's per-row setup was ~1.5 k of its
  // ~3.5 k cycles per row, profiles/r05/r5c/tl_als_new.log): bpre[j][f] = a_j[f] − Σ_{m>j} B_jm·h_m[f]
  // (the rows after j are still the old ones when row j is solved), rinv[j][f] = 1 / (B_jj + λ·DᵀD_ff),
  // and each row's Jacobi sweep count (0: the row takes the block PCR)
  {
    const double* sA = reinterpret_cast<const double*>(smem);
    const double* sH = sA + (size_t)k * F;
    const double* sB = sH + (size_t)k * F;
    double* bpre = reinterpret_cast<double*>(smem + als_pre_offset(F, k));
    double* rinv = bpre + (size_t)k * F;
    double* nswp = rinv + (size_t)k * F;
    for (int o = t; o < k * F; o += RED_NT) {
      const int j = o / F, f = o - j * F;
      double b = sA[o];
      for (int m = j + 1; m < k; ++m) b -= sB[j * k + m] * sH[m * F + f];
      bpre[o] = b;
      const double bjj = sB[j * k + j];
      rinv[o] = 1.0 / (bjj + lam * als_L_entry(F, f, f));
    }
    if (t < k) {
      const double bjj = sB[t * k + t];
      const double rho = 10.0 * lam / bjj;
      int nsw = 0;
      for (double r = 1.0; rho <= 0.05 && r > 0x1p-55; r *= rho) ++nsw;
      nswp[t] = (double)nsw;
    }
    __syncthreads();
    PH(3);
  }
  if (t < 64) {
    const int lane = t;
    double* sA = reinterpret_cast<double*>(smem);
    double* sH = sA + (size_t)k * F;
    double* sB = sH + (size_t)k * F;
    double* vb = sB + k * k;
    double* vx = vb + F;
    double* d0 = vx + F;
    double* e1 = d0 + F;
    double* e2 = e1 + F;
    double* vz = e2 + 4 * F;  // the block form's L0, L1, L2 are not used here
    int* idx = reinterpret_cast<int*>(vz + F) + 2 * F;
    const uint64_t lt = (1ull << lane) - 1ull;
    // λ·(DᵀD) entries of the lane's two features: the same for every row of the sweep
    double ld0[2], le1[2], le2[2], lm1[2], lm2[2];  // lm1/lm2: λ·L[f-1][f], λ·L[f-2][f]
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int f = 2 * lane + c;
      ld0[c] = f < F ? lam * als_L_entry(F, f, f) : 0.0;
      le1[c] = f + 1 < F ? lam * als_L_entry(F, f, f + 1) : 0.0;
      le2[c] = f + 2 < F ? lam * als_L_entry(F, f, f + 2) : 0.0;
      lm1[c] = (f < F && f >= 1) ? lam * als_L_entry(F, f - 1, f) : 0.0;
      lm2[c] = (f < F && f >= 2) ? lam * als_L_entry(F, f - 2, f) : 0.0;
    }
    double* bpre = reinterpret_cast<double*>(smem + als_pre_offset(F, k));
    const double* rinvp = bpre + (size_t)k * F;
    const double* nswp = rinvp + (size_t)k * F;
    for (int j = 0; j < k; ++j) {
      // the row's operands in one batch of LDS reads.  bpre[j] already holds a_j − Σ_{m>j} B_jm·h_m(old)
      // − Σ_{m<j} B_jm·h_m(new): the precompute subtracted the later rows (ascending m > j), each
      // earlier row its new values at its end (below, ascending m < j) — a different rounding order
      // from one sum over m != j for j >= 1 (the H-step agrees with scipy's sweep to ~1e-12 either
      // way, tests/test_gpu_als.py::test_h_step_matches_scipy_nnls at 1e-9)
      const double bjj = sB[j * k + j];
      const int nsw = (int)nswp[j];
      double hjv[2], bv[2], riv[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int f = 2 * lane + c;
        hjv[c] = f < F ? sH[j * F + f] : 0.0;
        bv[c] = f < F ? bpre[j * F + f] : 0.0;
        riv[c] = f < F ? rinvp[j * F + f] : 1.0;
      }
      double xnew[2] = {hjv[0], hjv[1]};  // an unused component (B_jj <= 0): row unchanged (oracle: same)
      if (bjj > 0.0) {
#ifdef CNMF_STAMPS
      const unsigned long long hs_t0 = __builtin_amdgcn_s_memtime();
      const unsigned long long hs_r0 = __builtin_amdgcn_s_memrealtime();
      int hs_iters = 0;
      unsigned long long hs_ph[4] = {0, 0, 0, 0}, hs_m = hs_t0;
      auto hs_mark = [&](int ph) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        hs_ph[ph] += now - hs_m;
        hs_m = now;
      };
#define HS_MARK(p) hs_mark(p)
#else
#define HS_MARK(p) ((void)0)
#endif
      // Jacobi (below) or the block PCR: decided per row from B_jj (the sweep count, precomputed)
      const bool jac = nsw > 0;
      double rb[2], rd[2], re1[2], re2[2], xf[2], rinv[2] = {1.0, 1.0};
      bool pas[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int f = 2 * lane + c;
        rb[c] = 0.0; rd[c] = 1.0; re1[c] = 0.0; re2[c] = 0.0; xf[c] = 0.0;
        pas[c] = false;
        const double hj = hjv[c];
        if (f < F) {
          rb[c] = bv[c];
          rinv[c] = riv[c];
          rd[c] = bjj + ld0[c];
          re1[c] = le1[c];
          re2[c] = le2[c];
          pas[c] = hj > 0.0;
          if (!jac) {  // the PCR's gathers read the row from LDS
            vb[f] = rb[c];
            d0[f] = rd[c];
            e1[f] = re1[c];
            e2[f] = re2[c];
          }
        }
        xf[c] = pas[c] ? hj : 0.0;  // warm start
      }
      int alpha = 3, beta = F + 1;  // BPP control (wave-uniform)
      // Jacobi: the row's Hessian M = B_jj·I + λ·DᵀD has off-diagonal row sums at most 10λ (the
      // |1, −4, −4, 1| of DᵀD) against a diagonal >= B_jj, so ρ = 10λ / B_jj bounds the Jacobi
      // contraction of any passive subsystem M_PP in the max norm.  At ρ <= 1/20 (B_jj is a sum over
      // all samples: ρ ~ 1e-4 at cfg5) sweeps from the warm start x = h_j reach the fp64 fixed
      // point in a few steps (bound: ρ^nsw <= 2^-55; exactly nsw sweeps run) —
      // the same solve as the block PCR below at a fraction of its per-row cost.
      HS_MARK(0);
      for (int iter = 0; iter < 5 * F + 10; ++iter) {
       if (jac) {
        // ---- M_PP x = b_P by Jacobi sweeps over the row's features (x = 0 off P); the neighbours
        // x[2l-2], x[2l-1] from lane l - 1 and x[2l+2], x[2l+3] from lane l + 1
        // exactly nsw sweeps, no per-sweep convergence ballot (round 5: the ballot's VALU -> SALU ->
        // branch round trip stalled every sweep; at cfg5's ρ ≈ 7e-5 the rows ran nsw = 5 sweeps anyway,
        // and a sweep at the fixed point changes no bit)
        const int nsw_s = __builtin_amdgcn_readfirstlane(nsw);
        for (int sw = 0; sw < nsw_s; ++sw) {
          const double p0 = dpp_wave_shr(xf[0]), p1 = dpp_wave_shr(xf[1]);
          const double n0 = dpp_wave_shl(xf[0]), n1 = dpp_wave_shl(xf[1]);
          double r0 = rb[0];
          r0 = fma(-lm1[0], p1, r0);
          r0 = fma(-re1[0], xf[1], r0);
          r0 = fma(-lm2[0], p0, r0);
          r0 = fma(-re2[0], n0, r0);
          double r1 = rb[1];
          r1 = fma(-lm1[1], xf[0], r1);
          r1 = fma(-re1[1], n0, r1);
          r1 = fma(-lm2[1], p1, r1);
          r1 = fma(-re2[1], n1, r1);
          const double x0 = pas[0] ? r0 * rinv[0] : 0.0;  // (pas is false past F)
          const double x1 = pas[1] ? r1 * rinv[1] : 0.0;
          xf[0] = x0;
          xf[1] = x1;
#ifdef CNMF_STAMPS
          hs_ph[1] += 1000ull;  // the stamps' "gather" slot counts the Jacobi sweeps (in thousands)
#endif
        }
        HS_MARK(2);
       } else {
        // ---- compress the passive set in feature order: idx[pos] = feature
        const uint64_t bal0 = __ballot(pas[0]), bal1 = __ballot(pas[1]);
        const int n = __popcll(bal0) + __popcll(bal1);
        const int pos0 = (int)__popcll(bal0 & lt) + (int)__popcll(bal1 & lt);
        const int pos[2] = {pos0, pos0 + (pas[0] ? 1 : 0)};
#pragma unroll
        for (int c = 0; c < 2; ++c)
          if (pas[c]) idx[pos[c]] = 2 * lane + c;
        lds_order();
        // ---- M_PP x = b_P by parallel cyclic reduction on 2x2 blocks (lane i = compressed rows
        // 2i, 2i+1; nb = ceil(n/2) <= 64 blocks; log2(nb) steps instead of n sequential LDLᵀ
        // steps).  The pentadiagonal M_PP is block tridiagonal: A_i (rows 2i, 2i+1 x columns 2i-2,
        // 2i-1), B_i (symmetric), C_i = A_{i+1}ᵀ.  Step s eliminates blocks i +- s:
        //   B_i -= A_i B_{i-s}⁻¹ A_iᵀ + C_i B_{i+s}⁻¹ C_iᵀ,  A_i <- -A_i B_{i-s}⁻¹ A_{i-s},
        //   d_i -= A_i B_{i-s}⁻¹ d_{i-s} + C_i B_{i+s}⁻¹ d_{i+s},  with C_i = A_{i+s}ᵀ at every
        // stride (the reduced systems are Schur complements of a symmetric matrix).  Positions >= n
        // are identity rows with zero coupling; blocks outside the wave contribute zero.
        {
          // compressed entry of position p: M_pp, M_p,p-1, M_p,p-2, b_p
          auto ent = [&](int p, double& m0, double& m1, double& m2, double& z) {
            m0 = 1.0; m1 = 0.0; m2 = 0.0; z = 0.0;
            if (p < n) {
              const int fp = idx[p];
              m0 = d0[fp];
              m1 = p >= 1 ? als_m_low(e1, e2, fp, idx[p - 1]) : 0.0;
              m2 = p >= 2 ? als_m_low(e1, e2, fp, idx[p - 2]) : 0.0;
              z = vb[fp];
            }
          };
          const int nb = (n + 1) >> 1;
          double p0m0, p0m1, p0m2, p0z, p1m0, p1m1, p1m2, p1z;
          ent(2 * lane, p0m0, p0m1, p0m2, p0z);
          ent(2 * lane + 1, p1m0, p1m1, p1m2, p1z);
          double b00 = p0m0, b01 = p1m1, b11 = p1m0;
          double a00 = p0m2, a01 = p0m1, a10 = 0.0, a11 = p1m2;
          double r0 = p0z, r1 = p1z;
#ifdef CNMF_STAMPS
          if (b00 + b11 + a00 + a11 + r0 + r1 == 12345.678) vb[0] = 0.0;  // the gathered entries landed
#endif
          HS_MARK(1);
          auto inv2 = [](double x00, double x01, double x11, double& i00, double& i01, double& i11) {
            const double det = fmax(fma(x00, x11, -x01 * x01), 1e-300);
            double id = __builtin_amdgcn_rcp(det);
            id = fma(id, fma(-det, id, 1.0), id);
            id = fma(id, fma(-det, id, 1.0), id);
            i00 = x11 * id;
            i11 = x00 * id;
            i01 = -x01 * id;
          };
          for (int st = 1; st < nb; st <<= 1) {
            double i00, i01, i11;
            inv2(b00, b01, b11, i00, i01, i11);
            const bool hl = lane >= st, hr = lane + st < 64;
            const int sl_ = hl ? lane - st : lane, sr_ = hr ? lane + st : lane;
            auto from = [&](double v, int src, bool ok) { const double u = __shfl(v, src, 64); return ok ? u : 0.0; };
            const double Li00 = from(i00, sl_, hl), Li01 = from(i01, sl_, hl), Li11 = from(i11, sl_, hl);
            const double La00 = from(a00, sl_, hl), La01 = from(a01, sl_, hl), La10 = from(a10, sl_, hl),
                         La11 = from(a11, sl_, hl), Lr0 = from(r0, sl_, hl), Lr1 = from(r1, sl_, hl);
            const double Ri00 = from(i00, sr_, hr), Ri01 = from(i01, sr_, hr), Ri11 = from(i11, sr_, hr);
            const double c00 = from(a00, sr_, hr), c10 = from(a01, sr_, hr), c01 = from(a10, sr_, hr),
                         c11 = from(a11, sr_, hr), Rr0 = from(r0, sr_, hr), Rr1 = from(r1, sr_, hr);
            // T = A_i B_{i-s}⁻¹, U = C_i B_{i+s}⁻¹
            const double t00 = fma(a00, Li00, a01 * Li01), t01 = fma(a00, Li01, a01 * Li11);
            const double t10 = fma(a10, Li00, a11 * Li01), t11 = fma(a10, Li01, a11 * Li11);
            const double u00 = fma(c00, Ri00, c01 * Ri01), u01 = fma(c00, Ri01, c01 * Ri11);
            const double u10 = fma(c10, Ri00, c11 * Ri01), u11 = fma(c10, Ri01, c11 * Ri11);
            b00 = b00 - fma(t00, a00, t01 * a01) - fma(u00, c00, u01 * c01);
            b01 = b01 - fma(t00, a10, t01 * a11) - fma(u00, c10, u01 * c11);
            b11 = b11 - fma(t10, a10, t11 * a11) - fma(u10, c10, u11 * c11);
            const double n00 = -fma(t00, La00, t01 * La10), n01 = -fma(t00, La01, t01 * La11);
            const double n10 = -fma(t10, La00, t11 * La10), n11 = -fma(t10, La01, t11 * La11);
            a00 = n00; a01 = n01; a10 = n10; a11 = n11;
            const double q0 = r0 - fma(t00, Lr0, t01 * Lr1) - fma(u00, Rr0, u01 * Rr1);
            const double q1 = r1 - fma(t10, Lr0, t11 * Lr1) - fma(u10, Rr0, u11 * Rr1);
            r0 = q0;
            r1 = q1;
          }
          double i00, i01, i11;
          inv2(b00, b01, b11, i00, i01, i11);
          if (2 * lane < n) vz[2 * lane] = fma(i00, r0, i01 * r1);
          if (2 * lane + 1 < n) vz[2 * lane + 1] = fma(i01, r0, i11 * r1);
        }
        lds_order();
        HS_MARK(2);
#pragma unroll
        for (int c = 0; c < 2; ++c) xf[c] = pas[c] ? vz[pos[c]] : 0.0;
        lds_order();
       }
        // the KKT check: x >= 0 on P, the dual y = (M x − b)_f >= 0 off P (neighbours outside the
        // row enter with zero coefficients), both from the x the sweep returns (the last
        // Jacobi sweep's residuals use the neighbours before that sweep's update — exact only once it
        // changed no bit; a cold start or a BPP flip far from the solution could misread a dual near 0)
        bool bad[2];
        {
          const double p0 = dpp_wave_shr(xf[0]), p1 = dpp_wave_shr(xf[1]);
          const double n0 = dpp_wave_shl(xf[0]), n1 = dpp_wave_shl(xf[1]);
          const double nm1[2] = {p1, xf[0]}, np1[2] = {xf[1], n0}, nm2[2] = {p0, p1}, np2[2] = {n0, n1};
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int f = 2 * lane + c;
            bad[c] = false;
            if (f < F) {
              const double x = xf[c];
              double y = rd[c] * x - rb[c];
              y += re1[c] * np1[c];
              y += lm1[c] * nm1[c];
              y += re2[c] * np2[c];
              y += lm2[c] * nm2[c];
              bad[c] = pas[c] ? x < 0.0 : y < 0.0;
            }
          }
        }
        const uint64_t bb0 = __ballot(bad[0]), bb1 = __ballot(bad[1]);
        const int ninf = __popcll(bb0) + __popcll(bb1);
        const int mb0 = bb0 ? 2 * (63 - __clzll(bb0)) : -1;
        const int mb1 = bb1 ? 2 * (63 - __clzll(bb1)) + 1 : -1;
        const int maxbad = mb0 > mb1 ? mb0 : mb1;
        int mode;
        if (ninf == 0) mode = 0;
        else if (ninf < beta) { beta = ninf; alpha = 3; mode = 1; }
        else if (alpha >= 1) { --alpha; mode = 1; }
        else mode = 2;
#ifdef CNMF_STAMPS
        ++hs_iters;
#endif
        HS_MARK(3);
        if (mode == 0) break;
#pragma unroll
        for (int c = 0; c < 2; ++c)
          if ((mode == 1 && bad[c]) || (mode == 2 && 2 * lane + c == maxbad)) pas[c] = !pas[c];
      }
#undef HS_MARK
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        xnew[c] = fmax(xf[c], 0.0);
        if (2 * lane + c < F) sH[j * F + 2 * lane + c] = xnew[c];
      }
#ifdef CNMF_STAMPS
      if (lane == 0 && hs_call < 64u && j < 4) {  // BPP iterations | the row's 100 MHz ticks << 16
        g_hs[(hs_call * 4 + j) * 2] = (unsigned long long)hs_iters | ((__builtin_amdgcn_s_memrealtime() - hs_r0) << 16);
        g_hs[(hs_call * 4 + j) * 2 + 1] = __builtin_amdgcn_s_memtime() - hs_t0;
#pragma unroll
        for (int q = 0; q < 4; ++q) g_hsp[(hs_call * 4 + j) * 4 + q] = hs_ph[q];
      }
#endif
      }
      // the later rows' right-hand sides take this row's new values (each lane its own features:
      // the later read is the same lane's, in order)
#pragma unroll
      for (int m = 1; m < ALS_MAX_K; ++m)  // k <= ALS_MAX_K (every ALS entry point checks it)
        if (m > j && m < k) {
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int f = 2 * lane + c;
            if (f < F) bpre[m * F + f] -= sB[m * k + j] * xnew[c];
          }
        }
      lds_order();
    }
  }
  __syncthreads();
  PH(4);
#ifdef CNMF_STAMPS
  if (t == 0 && blockIdx.x == 0) __hip_atomic_fetch_add(&g_hs_calls, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// the H-step sweep: one wave for F <= 128, else the workgroup form
__device__ __forceinline__ void als_hstep(unsigned char* smem, int F, int k, double lam, int t) {
  if (F <= 128) als_hstep_wave(smem, F, k, lam, t);
  else als_hstep_block(smem, F, k, lam, t);
}

// The W-step's passive-set table from HHᵀ (stride KP): per mask P the inverse of Q_PP,
// Q = HHᵀ + δ²11ᵀ, by Gauss-Jordan with partial pivoting, scattered to 4x4, and the valid flag.
// One wave, lane L = 4·mask + r holding row r of the 4x8 [Q | I] (rows / columns outside P at the
// identity): every lane eliminates its own row, so a pivot step is ~70 instructions for all 16
// masks instead of ~150 for one mask per lane (round 5: 1.9 -> ~0.5 µs of the ALS resume).  Rows
// are not moved: each lane carries its row's position, and a swap of positions c and piv only swaps
// the two lanes' position numbers.  The arithmetic is the row-per-thread form's, operation for
// operation: the pivot is the largest |a[pos][c]| over P's positions >= c, the first position on ties
// (the ascending strict-> search), the pivot row scaled by 1 / a[c][c], every other P row updated
// a[e] -= a[c] · pivot[e] — so the table is the same bits.
__device__ void als_table(const double* HHt, int KP, int k, double delta2, double* table, int t, int mstride = 16) {
  if (t < 64) {
    const int mask = t >> 2, r0 = t & 3;
    const int qb = t & ~3;  // the quad's first lane
    bool valid = !(k < 4 && (mask >> k) != 0);
    double a[8];
    double dmax = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool in = (mask >> r0 & 1) && (mask >> c & 1);
      const double q = (r0 < k && c < k) ? HHt[r0 * KP + c] + delta2 : 0.0;
      a[c] = in ? q : (r0 == c ? 1.0 : 0.0);
      a[4 + c] = r0 == c ? 1.0 : 0.0;
      if (in && r0 == c) dmax = fabs(q);
    }
    dmax = fmax(dmax, wt::dpp64<0xB1>(dmax));  // the quad's largest P diagonal (max: exact in any order)
    dmax = fmax(dmax, wt::dpp64<0x4E>(dmax));
    int pos = r0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (!(mask >> c & 1)) continue;  // identity column: nothing to eliminate (quad-uniform)
      const bool inp = (mask >> pos & 1) != 0;
      // the pivot: (|a[c]|, position) maximised lexicographically with the smaller position winning
      // ties, over P's positions >= c (position c always qualifies)
      double pv = (inp && pos >= c) ? fabs(a[c]) : -1.0;
      int pp = pos;
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const double ov = x == 0 ? wt::dpp64<0xB1>(pv) : wt::dpp64<0x4E>(pv);
        const int op = x == 0 ? __builtin_amdgcn_update_dpp(0, pp, 0xB1, 0xF, 0xF, true)
                              : __builtin_amdgcn_update_dpp(0, pp, 0x4E, 0xF, 0xF, true);
        const bool tk = ov > pv || (ov == pv && op < pp);
        pv = tk ? ov : pv;
        pp = tk ? op : pp;
      }
      valid = valid && pv > 1e-13 * dmax;
      // swap positions c and pp (position numbers only)
      const int npos = pos == pp ? c : (pos == c ? pp : pos);
      pos = npos;
      const bool piv = pos == c;
      if (piv) {
        const double inv = 1.0 / a[c];
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] *= inv;
      }
      // the pivot row to the quad: its lane is the one now at position c
      const unsigned long long pb = __ballot(piv);
      const int src = qb + (int)__builtin_ctzll((pb >> qb) & 0xFull);
      double pr[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) pr[e] = __shfl(a[e], src, 64);
      if (!piv && (mask >> pos & 1)) {
        const double fct = a[c];
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] -= fct * pr[e];
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool in = (mask >> pos & 1) && (mask >> c & 1);
      table[mask * mstride + pos * 4 + c] = (valid && in) ? a[4 + c] : 0.0;
    }
    if (r0 == 0) table[16 * mstride + mask] = valid ? 1.0 : 0.0;
  }
}

__global__ __launch_bounds__(RED_NT) void als_basis_kernel(const double* __restrict__ AB, double* __restrict__ H64,
                                                           double* __restrict__ Ht, double* __restrict__ HHt,
                                                           double* __restrict__ table, int F, int k, int KP,
                                                           double lam, double delta2, int do_update) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int t = threadIdx.x;
  const int V = F + k;
  if (do_update) {
    double* sA = reinterpret_cast<double*>(smem);
    double* sH = sA + (size_t)k * F;
    double* sB = sH + (size_t)k * F;
    for (int e = t; e < k * F; e += RED_NT) {
      sA[e] = AB[(e / F) * V + (e % F)];
      sH[e] = H64[e];
    }
    for (int e = t; e < k * k; e += RED_NT) sB[e] = AB[(e / k) * V + F + (e % k)];
    __syncthreads();
    als_hstep(smem, F, k, lam, t);
    for (int e = t; e < k * F; e += RED_NT) H64[e] = sH[e];
    __syncthreads();  // workgroup-scope fence + barrier: the H64 stores are visible to this workgroup
  }
  // Ht / HHt of the (new) H, then the passive-set table of the next W-step
  basis_update_block(nullptr, H64, Ht, HHt, F, k, KP, 0.0, 0.0, 0, nullptr, reinterpret_cast<double*>(smem));
  __syncthreads();
  als_table(HHt, KP, k, delta2, table, t);
}

// ------------------------------------------------------------------------------------------------
// Deterministic fp64 reduction of partials[n_parts][n_out]; optional fused basis update.
// grid = (ceil(n_out/64), nslice): block (c, s) sums rows of slice s for 64 outputs (<= 8 rows per
// thread, one batch of independent loads) and writes one stage row write-through (sc1); one lane
// per block then takes a ticket.  The block drawing the last ticket sums the stage rows with sc1
// loads in a fixed order — the hand-off needs no release/acquire fence (MI355X_MICROARCH.md,
// inter-workgroup visibility, "Valid forms" table row 1).
// ------------------------------------------------------------------------------------------------
struct UpdateArgs {
  double* H64;
  double* Ht;
  double* HHt;
  int F, k, KP;
  double l1, l2;
  double* stats;
};

constexpr int RED_ROWS_PER_THREAD = 8;

__global__ __launch_bounds__(RED_NT) void reduce_kernel(const double* __restrict__ partials,
                                                        int64_t n_parts, int n_out, int nslice,
                                                        double* __restrict__ stage,
                                                        uint32_t* __restrict__ counter,
                                                        double* __restrict__ out, int fuse,
                                                        UpdateArgs ua) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* red = reinterpret_cast<double*>(smem);        // [RED_NT]
  int* flag = reinterpret_cast<int*>(red + RED_NT);      // [4]
  double* upd = red + RED_NT + 2;                        // fused-update scratch

  const int t = threadIdx.x;
  const int l = t & 63;
  const int r = t >> 6;
  const int o = blockIdx.x * 64 + l;
  const int64_t lo = n_parts * blockIdx.y / nslice;
  const int64_t hi = n_parts * (blockIdx.y + 1) / nslice;
  double s = 0.0;
  if (o < n_out) {
    double v[RED_ROWS_PER_THREAD];
#pragma unroll
    for (int u = 0; u < RED_ROWS_PER_THREAD; ++u) {
      const int64_t b = lo + r + 4 * u;
      v[u] = b < hi ? partials[b * n_out + o] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < RED_ROWS_PER_THREAD; ++u) s += v[u];
  }
  red[t] = s;
  __syncthreads();
  if (r == 0 && o < n_out)
    __hip_atomic_store(stage + (size_t)blockIdx.y * n_out + o,
                       ((red[l] + red[64 + l]) + red[128 + l]) + red[192 + l], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  // the last slice of this 64-column block to arrive combines the block's slices (fixed order:
  // part r sums slices r, r+4, ...; the 4 parts in order)
  uint32_t* ccol = counter + CNT_RCOL0 + blockIdx.x;
  if (t == 0) {
    const uint32_t old = __hip_atomic_fetch_add(ccol, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = old == (uint32_t)nslice - 1;
  }
  __syncthreads();
  if (!flag[0]) return;
  {
    double v = 0.0;
    if (o < n_out) {
      double x[16];
      for (int s0 = r; s0 < nslice; s0 += 64) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int sl = s0 + 4 * u;
          x[u] = __hip_atomic_load(stage + (size_t)min(sl, nslice - 1) * n_out + o, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) v += s0 + 4 * u < nslice ? x[u] : 0.0;
      }
    }
    red[t] = v;
    __syncthreads();
    if (r == 0 && o < n_out) {
      const double sum = ((red[l] + red[64 + l]) + red[128 + l]) + red[192 + l];
      if (fuse)
        __hip_atomic_store(out + o, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        out[o] = sum;
    }
    if (t == 0) __hip_atomic_store(ccol, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!fuse) return;
  // every column block done -> the last one applies the basis update
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const uint32_t old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[1] = old == gridDim.x - 1;
  }
  __syncthreads();
  if (!flag[1]) return;
  if (t == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  double* ab = upd;
  for (int oo = t; oo < n_out; oo += RED_NT)
    ab[oo] = __hip_atomic_load(out + oo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  double* scratch = upd + ((n_out + 1) & ~1);
  basis_update_small(ab, ua.H64, ua.Ht, ua.HHt, ua.F, ua.k, ua.KP, ua.l1, ua.l2, 1, ua.stats,
                     scratch);  // fused only for KP = 4 (cnmf_reduce_update)
}

// One-level reduction for wide rows (n_out >= RW_MIN_OUT, e.g. cfg4's k(F+k) = 5056): workgroup c
// owns 16 columns; thread (rg, c) sums rows rg, rg + 16, ... (16 independent loads in flight per
// batch — ONE batch for <= 256 rows), then the 16 row groups in order through LDS.  No stage rows,
// ticket or second round trip: at 256 rows × 40 KB the two-level kernel above spent its 7.7 µs on
// its latency chain, not on the 10 MB it reads.  Fixed order: deterministic.
constexpr int RW_MIN_OUT = 1024, RW_MAX_ROWS = 1024;
template <int RW_COLS>
__global__ __launch_bounds__(RED_NT) void reduce_wide_kernel(const double* __restrict__ partials,
                                                             int64_t n_parts, int n_out,
                                                             double* __restrict__ out) {
  constexpr int RW_RG = RED_NT / RW_COLS;
  __shared__ double red[RW_RG][RW_COLS];
  const int t = threadIdx.x;
  const int c = t % RW_COLS, rg = t / RW_COLS;
  const int o = blockIdx.x * RW_COLS + c;
  double s = 0.0;
  if (o < n_out) {
    for (int64_t b0 = rg; b0 < n_parts; b0 += (int64_t)RW_RG * 16) {
      double x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int64_t b = b0 + (int64_t)RW_RG * u;
        x[u] = b < n_parts ? partials[b * n_out + o] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) s += x[u];
    }
  }
  red[rg][c] = s;
  __syncthreads();
  if (t < RW_COLS && o < n_out) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < RW_RG; ++q) v += red[q][t];
    out[o] = v;
  }
}

// ------------------------------------------------------------------------------------------------
// HBM read probe: the achievable streaming-read ceiling on this device (16-byte loads, 8 in flight
// per lane, grid-stride; one fp64 checksum per workgroup so nothing is dead code).
// ------------------------------------------------------------------------------------------------
#ifdef CNMF_DIAG
__global__ __launch_bounds__(256) void hbm_probe_kernel(const u32x4* __restrict__ buf, int64_t n16,
                                                        double* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  uint32_t acc = 0;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = SL_XLOAD(buf + i + u * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) {
    u32x4 v = buf[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  __shared__ uint32_t red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    for (int j = 0; j < 256; ++j) a ^= red[j];
    out[blockIdx.x] = (double)a;
  }
}
#endif

// ------------------------------------------------------------------------------------------------
// host side: kernel selection, occupancy-derived grid, launches
// ------------------------------------------------------------------------------------------------
using PassFn = const void*;

struct PassKernel {
  PassFn fn;
  int KP, NPW;
  bool split;
  size_t sx, sc;
};

template <typename TX, int KP, int FT, int NPW, bool SPLIT>
static PassKernel make_pk() {
  return PassKernel{reinterpret_cast<PassFn>(&mu_pass_kernel<TX, KP, FT, NPW, SPLIT>), KP, NPW, SPLIT,
                    sizeof(TX), sizeof(typename Compute<TX>::T)};
}

template <typename TX, int FT, int NPW, bool SPLIT>
static PassKernel make_pk_als() {
  return PassKernel{reinterpret_cast<PassFn>(&mu_pass_kernel<TX, 4, FT, NPW, SPLIT, true>), 4, NPW, SPLIT,
                    sizeof(TX), sizeof(typename Compute<TX>::T)};
}

// the constrained-ALS W-step pass (k <= 4): the VALU pass kernel with the ALS phase 2 and fp64 Ht
template <typename TX>
static bool pick_als_tx(int F, int np, PassKernel* out) {
  if (F == 81 && np == 2) { *out = make_pk_als<TX, 81, 2, true>(); return true; }  // IOP grid (cfg5)
  if (np <= 1) { *out = make_pk_als<TX, 0, 1, true>(); return true; }
  if (np == 2) { *out = make_pk_als<TX, 0, 2, true>(); return true; }
  const int npw = (np + NWAVE - 1) / NWAVE;
  if (npw <= 2) { *out = make_pk_als<TX, 0, 2, false>(); return true; }
  if (npw <= 4) { *out = make_pk_als<TX, 0, 4, false>(); return true; }
  return false;
}

template <typename TX, int KP>
static bool pick_kp(int F, int np, PassKernel* out) {
  if (F == 81 && np == 2) { *out = make_pk<TX, KP, 81, 2, true>(); return true; }  // IOP grid
  if (np <= 1) { *out = make_pk<TX, KP, 0, 1, true>(); return true; }
  if (np == 2) { *out = make_pk<TX, KP, 0, 2, true>(); return true; }
  const int npw = (np + NWAVE - 1) / NWAVE;
  if (npw <= 1) { *out = make_pk<TX, KP, 0, 1, false>(); return true; }
  if (npw <= 2) { *out = make_pk<TX, KP, 0, 2, false>(); return true; }
  if (npw <= 4) { *out = make_pk<TX, KP, 0, 4, false>(); return true; }
  return false;
}

template <typename TX>
static bool pick_tx(int KP, int F, int np, PassKernel* out) {
  switch (KP) {
    case 4: return pick_kp<TX, 4>(F, np, out);
    case 8: return pick_kp<TX, 8>(F, np, out);
    case 16: return pick_kp<TX, 16>(F, np, out);
  }
  return false;
}

template <typename TX, int KP>
static PassKernel make_mfma(int) {
  return PassKernel{reinterpret_cast<PassFn>(&mu_pass_mfma_kernel<TX, KP, 81>), KP, 0, true,
                    sizeof(TX), sizeof(float)};
}

// The matrix-core pass serves fp32 / bf16 X on the compile-time IOP grid (F = 81, V <= 97);
// other widths take mu_pass_kernel (its runtime-F MFMA form spilled registers).
static bool pick_mfma(int x_dtype, int F, int k, PassKernel* out) {
  if (F != 81 || F + k > 16 * NB_MAX || (x_dtype != CNMF_F32 && x_dtype != CNMF_BF16)) return false;
  const int KP = k <= 4 ? 4 : (k <= 8 ? 8 : 16);
  const bool bf = x_dtype == CNMF_BF16;
  switch (KP) {
    case 4: *out = bf ? make_mfma<bf16_t, 4>(F) : make_mfma<float, 4>(F); return true;
    case 8: *out = bf ? make_mfma<bf16_t, 8>(F) : make_mfma<float, 8>(F); return true;
    default: *out = bf ? make_mfma<bf16_t, 16>(F) : make_mfma<float, 16>(F); return true;
  }
}

static int padded_k(int k) { return k <= 4 ? 4 : (k <= 8 ? 8 : 16); }

static constexpr size_t kMaxLds = 160 * 1024;
// A/B switches for benchmarking: CNMF_PASS_KERNEL=valu|mfma|sl restricts the accumulating pass to
// one kernel family (CNMF_FORCE_VALU=1 is the older spelling of "valu")
static const char* pass_choice() {
  const char* e = diag_env("CNMF_PASS_KERNEL");
  if (e && *e) return e;
  return diag_env("CNMF_FORCE_VALU") ? "valu" : "";
}
static bool g_force_valu = strcmp(pass_choice(), "valu") == 0;
static bool g_no_sl = strcmp(pass_choice(), "valu") == 0 || strcmp(pass_choice(), "mfma") == 0;

// the sample-lane pass serves the headline shape: fp32 X, F = 81, k = 4 (full tiles)
static bool use_sl(int x_dtype, int F, int k) {
  return !g_no_sl && x_dtype == CNMF_F32 && F == sl::F && k == sl::K;
}

// the bf16 matrix-core pass (§8 a8): bf16 X, 9 <= k <= 16, F % 4 == 0 (8-byte aligned rows for the
// transposed LDS reads), F <= 64·NBW_MAX
static bool use_bf16_mfma(int x_dtype, int F, int k) {
  return x_dtype == CNMF_BF16 && k >= 9 && k <= 16 && F % 4 == 0 && F <= 64 * bm::NBW_MAX &&
         bm::lds(F).total <= (int)(160 * 1024);
}

// the wave-tile bf16 pass (mu_pass_bfw_kernel) serves the accumulating / updating passes of the
// bf16 matrix-core shapes over their full 64-sample tiles (the ragged tail: one workgroup of
// mu_pass_bf16_mfma_kernel); CNMF_BFW=0 (diagnostic build) keeps the 64-sample kernel for A/B runs
static bool g_no_bfw = diag_env("CNMF_BFW") && atoi(diag_env("CNMF_BFW")) == 0;
static bool use_bfw(int x_dtype, int F, int k) {
  return !g_no_bfw && !g_force_valu && use_bf16_mfma(x_dtype, F, k) && F >= 8 && F <= 16 * bw::NBX &&
         k * (F + k) >= 1024 && bw::lds(F).total <= (int)kMaxLds;
}
static PassFn bfw_fn(int F, int k) {
#ifdef CNMF_DIAG  // CNMF_BFW_HTERMS=2: phase 1 with H in two bf16 terms (round-6 experiment, not kept)
  if (bm::ksteps(F) == 10 && k == 16 && diag_env("CNMF_BFW_HTERMS") && atoi(diag_env("CNMF_BFW_HTERMS")) == 2)
    return reinterpret_cast<PassFn>(&mu_pass_bfw_kernel<10, 16, 2>);
#endif
  return (bm::ksteps(F) == 10 && k == 16) ? reinterpret_cast<PassFn>(&mu_pass_bfw_kernel<10, 16>)
                                          : reinterpret_cast<PassFn>(&mu_pass_bfw_kernel<0, 0>);
}

static int select_pass(int x_dtype, int F, int k, PassKernel* pk, size_t* lds, bool mfma_ok = true) {
  if (F < 1 || k < 1) return set_err(CNMF_ERR_SHAPE, "invalid shape F=%d k=%d", F, k);
  if (k > 16) return set_err(CNMF_ERR_UNSUPPORTED, "k=%d > 16 is not supported", k);
  if (mfma_ok && !g_force_valu && use_bf16_mfma(x_dtype, F, k)) {
    *pk = PassKernel{reinterpret_cast<PassFn>(&mu_pass_bf16_mfma_kernel), 16, 0, true, 2, 4};
    *lds = (size_t)bm::lds(F).total;
    return CNMF_OK;
  }
  const int KP = padded_k(k);
  const int np = (F + k + 63) / 64;
  bool ok = mfma_ok && !g_force_valu && pick_mfma(x_dtype, F, k, pk);
  if (!ok) switch (x_dtype) {
    case CNMF_F32: ok = pick_tx<float>(KP, F, np, pk); break;
    case CNMF_F64: ok = pick_tx<double>(KP, F, np, pk); break;
    case CNMF_BF16: ok = pick_tx<bf16_t>(KP, F, np, pk); break;
    default: return set_err(CNMF_ERR_ARG, "unknown x_dtype %d", x_dtype);
  }
  if (!ok) return set_err(CNMF_ERR_UNSUPPORTED, "n_features=%d too wide for the pass kernel", F);
  *lds = pass_lds(F, KP, pk->sx, pk->sc).total;
  if (*lds > kMaxLds)
    return set_err(CNMF_ERR_UNSUPPORTED, "n_features=%d needs %zu B of LDS per tile (> %zu)", F, *lds,
                   kMaxLds);
  return CNMF_OK;
}

struct OccKey {
  int dev;
  PassFn fn;
  size_t lds;
  bool operator==(const OccKey& o) const { return dev == o.dev && fn == o.fn && lds == o.lds; }
};
struct OccHash {
  size_t operator()(const OccKey& k) const {
    return std::hash<const void*>()(k.fn) ^ (k.lds * 1315423911u) ^ (size_t)k.dev;
  }
};
static std::mutex g_occ_mu;
static std::unordered_map<OccKey, int64_t, OccHash> g_occ;

// max co-resident workgroups of this kernel on the current device (occupancy × CUs), cached
static int64_t max_resident(PassFn fn, size_t lds) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  OccKey key{dev, fn, lds};
  {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto it = g_occ.find(key);
    if (it != g_occ.end()) return it->second;
  }
  // the function's LDS ceiling at the chip's maximum, not at this plan's size: a later plan of the
  // same kernel with a smaller (cached) size must not lower it under an earlier, larger one
  if (lds > 64 * 1024)
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds) != hipSuccess)
      return -1;
  int per_cu = 0, ncu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, lds) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  // MI355X_MICROARCH.md "Correctness boundaries": the occupancy API reports one block per CU too
  // many for kernels of 81-112 SGPRs; every kernel here stays <= 112, whose residency is
  // min(API, 8, floor(800 / (112 + 16))) = at most 6 256-thread blocks per CU
  per_cu = std::min(per_cu, std::min(8, 800 / (112 + 16)));
  if (per_cu < 1) return 0;
  int64_t v = (int64_t)per_cu * ncu;
  std::lock_guard<std::mutex> lk(g_occ_mu);
  g_occ[key] = v;
  return v;
}

// the persistent cfg4 launch (mu_iter_bfw_kernel): bf16 X, F with 10 K-steps (289..320), k = 16,
// whole 64-sample tiles, >= 6 wave-tile pairs' worth of tiles per workgroup (the prefetch of the
// next iteration's first pair must find its W' retired), the grid co-resident.  Layout 6 only (the
// per-iteration launches, layout 4, were faster on the MI355X measured: DESIGN §3.4).
struct BwpLaunch {
  int64_t G, n_tiles;
  size_t lds;
};
static bool bwp_plan(int64_t n_rows, int x_dtype, int F, int k, int layout, BwpLaunch* out) {
  if (layout != 6) return false;  // opt-in: MUPlan.tune() times it against the per-iteration launches
  if (!use_bfw(x_dtype, F, k) || bm::ksteps(F) != 10 || k != 16 || n_rows <= 0 || n_rows % TS != 0) return false;
  const size_t lds = (size_t)bw::lds(F).total + align16((size_t)k * F * 8) + 16;
  if (lds > kMaxLds) return false;
  const int64_t n_tiles = n_rows / TS;
  const int64_t cap = max_resident(reinterpret_cast<PassFn>(&mu_iter_bfw_kernel), lds);
  int64_t G = std::min<int64_t>(cap, n_tiles / 7);
  if (G < 1) return false;
  const int64_t rounds = (n_tiles + G - 1) / G;  // >= 7: every workgroup >= 6 tiles
  G = (n_tiles + rounds - 1) / rounds;
  *out = BwpLaunch{G, n_tiles, lds};
  return true;
}

static int64_t pass_grid(int64_t n_rows, PassFn fn, size_t lds) {
  const int64_t n_tiles = (n_rows + TS - 1) / TS;
  if (n_tiles == 0) return 0;
  const int64_t maxb = max_resident(fn, lds);
  if (maxb <= 0) return -1;
  const int64_t rounds = (n_tiles + maxb - 1) / maxb;
  return (n_tiles + rounds - 1) / rounds;
}

static size_t reduce_lds(int n_out, int fuse, int F, int k) {
  size_t d = RED_NT + 2;
  if (fuse) d += ((size_t)(n_out + 1) & ~size_t(1)) + update_lds_doubles(F, k, padded_k(k));
  return d * sizeof(double);
}

// ------------------------------------------------------------------------------------------------
// GPU NNDSVD initialisation (sklearn's _initialize_nmf SK:317-373 over
// randomized_svd, extmath.py:530-604).  sklearn's range finder alternates Q <- lu(X·Q),
// Q <- lu(Xᵀ·Q): only span(Q) matters to the result (U, s, Vt are invariant under an orthonormal
// change of basis of the range; svd_flip fixes the signs), and span(Xᵀ·X·Q) needs only the F × F
// Gram matrix C = XᵀX.  So the device does the work that scales with N:
//   ig_gram_kernel    C = XᵀX and the column sums of X (fp64, per-workgroup partial rows, reduced by
//                     cnmf_reduce_partials) — one pass over X;
//   ig_xm_kernel      U = X·M (M = F × k from the small host algebra), fp64 — one pass over X;
//   ig_stats_kernel   per column of U: Σ max(u,0)², Σ min(u,0)², and the first entry of largest |u|
//                     (svd_flip's u-based sign) — per-workgroup rows;
//   ig_fill_kernel    W from U: sqrt(S0)|u| (j = 0) or lbd·part(sign·u)/‖part‖, < eps -> 0, and the
//                     nndsvda fill — in X's dtype;
// while the host does sklearn's F × r / r × r algebra in fp64 (cnmf_amd/gpu_init.py).
// ------------------------------------------------------------------------------------------------
namespace ig {
constexpr int FP = 96;   // features padded (F <= 96)
constexpr int GT = 64;   // rows per staged tile
constexpr int KMAX = 16;
}  // namespace ig

// C = XᵀX (F × F) and colsum (F) of this workgroup's rows [r0, r1): thread (a, c) owns C rows
// 3a..3a+2 × columns 12c..12c+11 (fp64 registers); the tile is staged in LDS as fp64 [GT][FP].
// Output row: [F·F | F].
template <typename TX>
__global__ __launch_bounds__(256) void ig_gram_kernel(const TX* __restrict__ X, int64_t n_rows, int F,
                                                      int64_t rows_per_block, double* __restrict__ partials) {
  using namespace ig;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* tile = reinterpret_cast<double*>(smem);  // [GT][FP]
  const int t = threadIdx.x;
  const int a = t >> 3, c = t & 7;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n_rows ? r0 + rows_per_block : n_rows;
  double acc[3][12], cs[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    cs[i] = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) acc[i][j] = 0.0;
  }
  for (int64_t rt = r0; rt < r1; rt += GT) {
    const int nr = (int)(r1 - rt < GT ? r1 - rt : GT);
    __syncthreads();
    for (int e = t; e < GT * FP; e += 256) {
      const int r = e / FP, f = e - r * FP;
      tile[e] = (r < nr && f < F) ? (double)to_c(*(X + (rt + r) * F + f)) : 0.0;
    }
    __syncthreads();
    for (int r = 0; r < nr; ++r) {
      const double* row = tile + r * FP;
      double xa[3], xb[12];
#pragma unroll
      for (int i = 0; i < 3; ++i) xa[i] = row[3 * a + i];
#pragma unroll
      for (int j = 0; j < 12; ++j) xb[j] = row[12 * c + j];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 12; ++j) acc[i][j] = fma(xa[i], xb[j], acc[i][j]);
        cs[i] += xa[i];
      }
    }
  }
  double* prow = partials + (size_t)blockIdx.x * (F * F + F);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int fi = 3 * a + i;
    if (fi >= F) continue;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const int fj = 12 * c + j;
      if (fj < F) prow[fi * F + fj] = acc[i][j];
    }
    if (c == 0) prow[F * F + fi] = cs[i];
  }
}

// U[n][j] = Σ_f X[n][f]·M[f][j] (fp64), k <= 16: thread = (row of the tile, component group)
template <typename TX>
__global__ __launch_bounds__(256) void ig_xm_kernel(const TX* __restrict__ X, int64_t n_rows, int F, int k,
                                                    const double* __restrict__ M, double* __restrict__ U) {
  using namespace ig;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sM = reinterpret_cast<double*>(smem);  // [F][k]
  float* tile = reinterpret_cast<float*>(smem + (size_t)FP * KMAX * 8);  // [GT][F + 1] (fp32 copy; exact for f32/bf16)
  double* tile64 = reinterpret_cast<double*>(smem + (size_t)FP * KMAX * 8);  // f64 X: [GT][F + 1]
  const int t = threadIdx.x;
  for (int e = t; e < F * k; e += 256) sM[e] = M[e];
  const int r = t & (GT - 1), jg = t >> 6;  // 4 component groups: j = jg, jg + 4, ...
  const int64_t n_tiles = (n_rows + GT - 1) / GT;
  for (int64_t tb = blockIdx.x; tb < n_tiles; tb += gridDim.x) {
    const int64_t row0 = tb * GT;
    const int nr = (int)(n_rows - row0 < GT ? n_rows - row0 : GT);
    __syncthreads();
    for (int e = t; e < nr * F; e += 256) {
      const int rr = e / F, f = e - rr * F;
      if (std::is_same<TX, double>::value)
        tile64[rr * (F + 1) + f] = (double)to_c(*(X + row0 * F + e));
      else
        tile[rr * (F + 1) + f] = (float)to_c(*(X + row0 * F + e));
    }
    __syncthreads();
    if (r < nr) {
      for (int j = jg; j < k; j += 4) {
        double u = 0.0;
        for (int f = 0; f < F; ++f) {
          const double x = std::is_same<TX, double>::value ? tile64[r * (F + 1) + f] : (double)tile[r * (F + 1) + f];
          u = fma(x, sM[f * k + j], u);
        }
        U[(row0 + r) * k + j] = u;
      }
    }
  }
}

// per column j of U (N × k fp64) over this workgroup's rows: [Σ max(u,0)², Σ min(u,0)², max|u|,
// the u at the first row attaining it, that row] — 5 doubles per column
__global__ __launch_bounds__(256) void ig_stats_kernel(const double* __restrict__ U, int64_t n_rows, int k,
                                                       int64_t rows_per_block, double* __restrict__ out) {
  __shared__ double red[256][5];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n_rows ? r0 + rows_per_block : n_rows;
  for (int j = 0; j < k; ++j) {
    double sp = 0.0, sn = 0.0, mx = -1.0, mv = 0.0, mi = 0.0;
    for (int64_t r = r0 + t; r < r1; r += 256) {  // rows ascending per thread: first max kept
      const double u = U[r * k + j];
      if (u > 0.0) sp = fma(u, u, sp);
      if (u < 0.0) sn = fma(u, u, sn);
      if (fabs(u) > mx) {
        mx = fabs(u);
        mv = u;
        mi = (double)r;
      }
    }
    red[t][0] = sp;
    red[t][1] = sn;
    red[t][2] = mx;
    red[t][3] = mv;
    red[t][4] = mi;
    __syncthreads();
    if (t == 0) {  // fixed order; ties on |u|: the lowest row (np.argmax's first occurrence)
      double a0 = 0.0, a1 = 0.0, bm = -1.0, bv = 0.0, bi = 0.0;
      for (int i = 0; i < 256; ++i) {
        a0 += red[i][0];
        a1 += red[i][1];
        if (red[i][2] > bm || (red[i][2] == bm && red[i][4] < bi)) {
          bm = red[i][2];
          bv = red[i][3];
          bi = red[i][4];
        }
      }
      double* o = out + ((size_t)blockIdx.x * k + j) * 5;
      o[0] = a0;
      o[1] = a1;
      o[2] = bm;
      o[3] = bv;
      o[4] = bi;
    }
    __syncthreads();
  }
}

// W[n][j] from U[n][j]: v = coef_j · part_j(sign_j · u) with part 0 = |u|, 1 = max(u,0), 2 = |min(u,0)|;
// v < eps -> 0; then v == 0 -> fill (nndsvda: X.mean(); nndsvd / nndsvdar: 0)
template <typename TW>
__global__ __launch_bounds__(256) void ig_fill_kernel(const double* __restrict__ U, int64_t n, int k,
                                                      const double* __restrict__ coef, const int* __restrict__ part,
                                                      const double* __restrict__ sgn, double eps, double fill,
                                                      TW* __restrict__ W) {
  const int64_t total = n * k;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int j = (int)(e % k);
    const double u = sgn[j] * U[e];
    const int pj = part[j];
    const double p = pj == 0 ? fabs(u) : (pj == 1 ? (u > 0.0 ? u : 0.0) : (u < 0.0 ? -u : 0.0));
    double v = pj == 0 ? coef[j] * p : p * coef[j];
    if (v < eps) v = 0.0;
    if (v == 0.0) v = fill;
    W[e] = (TW)v;
  }
}

}  // namespace cnmf

using namespace cnmf;


// ------------------------------------------------------------------------------------------------
// Weighted / masked MU (spec + oracle: oracle/wmu_ref.py).  Per-element
// weights M >= 0 (0 = a missing value, 1/σ² = an uncertainty weight):
//   W <- W ∘ ((M∘X)·Hᵀ) / ((M∘(W·H))·Hᵀ)        H <- H ∘ (W'ᵀ·(M∘X)) / (W'ᵀ·(M∘(W'·H)))
// in the order of SK:831-870 (W-step first; the H-step uses the new W'), zero denominators ->
// EPS32 as SK:620/706.  With M = 1 both reduce to SK's Frobenius MU.
//
// One HBM pass per iteration: X and M once (8 bytes per element) plus W read + written.  Unlike
// the unweighted update the W denominator does not factor through HHᵀ (M couples the features),
// so phase 1 forms the reconstruction w·h_f per element.  Per tile of `ts` samples (staged in LDS):
//   phase 1  P = 256/ts lanes per sample, features strided by P (consecutive lanes -> consecutive
//            features), fp64: rec = w·h_f, num_j += m·x·h_jf, den_j += m·rec·h_jf; xor-shuffle
//            sums over the P lanes; the part-0 lane writes w' (HBM and LDS)
//   phase 2  thread = feature: over the tile's samples rec' = w'·h_f, A_j += w'_j·m·x,
//            D_j += w'_j·m·rec' in fp32, folded into fp64 registers once per tile
// Each workgroup writes one fp64 row [A | D] (2kF) at the end; cnmf_reduce_partials sums the rows
// in fixed order and cnmf_wmu_basis_update applies the H-step.  Loss pass: Σ m·(x − w·h)² in fp64.
// Limits: k <= 8, F <= 512 (registers of phase 2: NFT features per thread).
// ------------------------------------------------------------------------------------------------
constexpr int WMU_CH = 5;    // features per fp32 chain in phase 1
constexpr int WMU_MAXC = 8;  // 16-byte chunks per thread and array of one tile (ts·F <= 8192)
template <int KP, int NFT>
__global__ __launch_bounds__(NT) void wmu_pass_kernel(const float* __restrict__ X, const float* __restrict__ M,
                                                      float* __restrict__ W, const double* __restrict__ H64,
                                                      double* __restrict__ partials, int64_t n_rows, int F,
                                                      int k, int ts, int flags, int64_t n_tiles, int rows) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* sX = reinterpret_cast<float*>(smem);  // [ts][F]
  float* sM = sX + ts * F;                     // [ts][F]
  float* sHt = sM + ts * F;                    // [F][KP] (columns >= k zero)
  float* sWn = sHt + KP * F;                   // [ts][KP] the tile's new W
  float* sW = sWn + ts * KP;                   // [ts][k] the tile's W (staged with X and M)
  double* sRed = reinterpret_cast<double*>(smem + ((size_t)(2 * ts * F + KP * F + 2 * ts * KP) * 4 + 15) / 16 * 16);
  const int t = threadIdx.x;
  const int lane = t & 63;
  const bool do_loss = (flags & CNMF_PASS_LOSS) != 0;
  const bool do_upd = (flags & CNMF_PASS_UPDATE_W) != 0;
  const bool do_acc = (flags & CNMF_PASS_ACCUMULATE) != 0;
  const int P = NT / ts;  // lanes per sample in phase 1 (a power of two <= 64)
  const int sp = t / P;
  const int part = t - sp * P;
  for (int e = t; e < KP * F; e += NT) {
    const int f = e / KP, j = e - f * KP;
    sHt[e] = j < k ? (float)H64[j * F + f] : 0.f;
  }
  __syncthreads();
  // phase-2 threads: F <= 256: G2 = 256/F groups of F threads, group g takes the samples g, g+G2, ..;
  // F > 256: one group, features t and t + 256.  Each group writes its own fp64 row.
  const int G2 = NFT == 1 ? NT / F : 1;
  const int g2 = NFT == 1 ? t / F : 0;
  const int fb = NFT == 1 ? t - g2 * F : t;
  float hf[NFT][KP];
  double A64[NFT][KP], D64[NFT][KP];
#pragma unroll
  for (int u = 0; u < NFT; ++u) {
    const int f = fb + NT * u;
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      hf[u][j] = (g2 < G2 && f < F) ? sHt[f * KP + j] : 0.f;
      A64[u][j] = 0.0;
      D64[u][j] = 0.0;
    }
  }
  double loss = 0.0;
  // the next tile's X and M ride in registers (16-byte loads of the tile's contiguous span) while
  // this tile computes; a span whose length is not a multiple of 16 bytes (only a ragged last
  // tile) stages its tail with 4-byte loads
  u32x4 px[WMU_MAXC], pm[WMU_MAXC], pw;
  auto load_tile = [&](int64_t tile) {
    const int64_t r0 = tile * ts;
    const int nsr = (int)min<int64_t>(ts, n_rows - r0);
    const int nch = nsr * F / 4;
    const u32x4* x4 = reinterpret_cast<const u32x4*>(X + r0 * F);
    const u32x4* m4 = reinterpret_cast<const u32x4*>(M + r0 * F);
    if (t < nsr * k / 4) pw = reinterpret_cast<const u32x4*>(W + r0 * k)[t];  // the tile's W span
#pragma unroll
    for (int c = 0; c < WMU_MAXC; ++c) {
      const int i = t + NT * c;
      if (i < nch) {
        px[c] = __builtin_nontemporal_load(x4 + i);
        pm[c] = __builtin_nontemporal_load(m4 + i);
      }
    }
  };
  if ((int64_t)blockIdx.x < n_tiles) load_tile(blockIdx.x);
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t r0 = tile * ts;
    const int ns = (int)min<int64_t>(ts, n_rows - r0);
    __syncthreads();  // the previous tile's phase 2 is done with sX / sM / sWn
    {
      const int nch = ns * F / 4;
#pragma unroll
      for (int c = 0; c < WMU_MAXC; ++c) {
        const int i = t + NT * c;
        if (i < nch) {
          reinterpret_cast<u32x4*>(sX)[i] = px[c];
          reinterpret_cast<u32x4*>(sM)[i] = pm[c];
        }
      }
      for (int e = 4 * nch + t; e < ns * F; e += NT) {
        sX[e] = X[r0 * F + e];
        sM[e] = M[r0 * F + e];
      }
      if (t < ns * k / 4) reinterpret_cast<u32x4*>(sW)[t] = pw;
      for (int e = ns * k / 4 * 4 + t; e < ns * k; e += NT) sW[e] = W[r0 * k + e];
    }
    if (tile + gridDim.x < n_tiles) load_tile(tile + gridDim.x);
    __syncthreads();
    // ---- phase 1
    {
      const bool valid = sp < ns;
      double w[KP];
#pragma unroll
      for (int j = 0; j < KP; ++j) w[j] = (valid && j < k) ? (double)sW[sp * k + j] : 0.0;
      double num[KP], den[KP], l = 0.0;
#pragma unroll
      for (int j = 0; j < KP; ++j) num[j] = den[j] = 0.0;
      if (valid) {
        const float* xr = sX + sp * F;
        const float* mr = sM + sp * F;
        if (do_loss) {
          for (int f = part; f < F; f += P) {
            double rec = 0.0;
#pragma unroll
            for (int j = 0; j < KP; ++j) rec = fma(w[j], (double)sHt[f * KP + j], rec);
            const double r = (double)xr[f] - rec;
            l = fma((double)mr[f] * r, r, l);
          }
        } else {
          // fp32 chains of WMU_CH features folded into fp64 (the precision note of phase12)
          float w32[KP];
#pragma unroll
          for (int j = 0; j < KP; ++j) w32[j] = (float)w[j];
          for (int f0 = part; f0 < F; f0 += WMU_CH * P) {
            float nc[KP], dc[KP];
#pragma unroll
            for (int j = 0; j < KP; ++j) nc[j] = dc[j] = 0.f;
#pragma unroll
            for (int c = 0; c < WMU_CH; ++c) {
              const int f = f0 + c * P;
              if (f < F) {
                float h[KP];
#pragma unroll
                for (int j = 0; j < KP; j += 4) {
                  const float4 v = *reinterpret_cast<const float4*>(sHt + f * KP + j);
                  h[j] = v.x;
                  h[j + 1] = v.y;
                  h[j + 2] = v.z;
                  h[j + 3] = v.w;
                }
                float rec = 0.f;
#pragma unroll
                for (int j = 0; j < KP; ++j) rec = fmaf(w32[j], h[j], rec);
                const float m = mr[f];
                const float mx = m * xr[f], mrec = m * rec;
#pragma unroll
                for (int j = 0; j < KP; ++j) {
                  nc[j] = fmaf(mx, h[j], nc[j]);
                  dc[j] = fmaf(mrec, h[j], dc[j]);
                }
              }
            }
#pragma unroll
            for (int j = 0; j < KP; ++j) {
              num[j] += (double)nc[j];
              den[j] += (double)dc[j];
            }
          }
        }
      }
      for (int off = 1; off < P; off <<= 1) {  // the sample's P lanes are consecutive
        l += __shfl_xor(l, off);
#pragma unroll
        for (int j = 0; j < KP; ++j) {
          num[j] += __shfl_xor(num[j], off);
          den[j] += __shfl_xor(den[j], off);
        }
      }
      if (do_loss) {
        if (part == 0 && valid) loss += l;
      } else if (part == 0 && sp < ts) {
#pragma unroll
        for (int j = 0; j < KP; ++j) {
          float wn = 0.f;
          if (valid && j < k) {
            if (do_upd) {
              double d = den[j];
              if (d == 0.0) d = EPS32;  // SK:620
              wn = (float)(w[j] * (num[j] / d));
              W[(r0 + sp) * k + j] = wn;
            } else {
              wn = (float)w[j];
            }
          }
          sWn[sp * KP + j] = wn;
        }
      }
    }
    if (!do_acc) continue;
    __syncthreads();
    // ---- phase 2
#pragma unroll
    for (int u = 0; u < NFT; ++u) {
      const int f = fb + NT * u;
      if (g2 < G2 && f < F) {
        float a32[KP], d32[KP];
#pragma unroll
        for (int j = 0; j < KP; ++j) a32[j] = d32[j] = 0.f;
#pragma unroll 4
        for (int s2 = g2; s2 < ns; s2 += G2) {
          const float x = sX[s2 * F + f];
          const float m = sM[s2 * F + f];
          float wr[KP];
#pragma unroll
          for (int j = 0; j < KP; j += 4) {
            const float4 v = *reinterpret_cast<const float4*>(sWn + s2 * KP + j);
            wr[j] = v.x;
            wr[j + 1] = v.y;
            wr[j + 2] = v.z;
            wr[j + 3] = v.w;
          }
          float rec = 0.f;
#pragma unroll
          for (int j = 0; j < KP; ++j) rec = fmaf(wr[j], hf[u][j], rec);
          const float mx = m * x, mrec = m * rec;
#pragma unroll
          for (int j = 0; j < KP; ++j) {
            a32[j] = fmaf(wr[j], mx, a32[j]);
            d32[j] = fmaf(wr[j], mrec, d32[j]);
          }
        }
#pragma unroll
        for (int j = 0; j < KP; ++j) {
          A64[u][j] += (double)a32[j];
          D64[u][j] += (double)d32[j];
        }
      }
    }
  }
  if (do_loss) {  // the workgroup's Σ: waves by shuffles, then the 4 wave sums in order
    for (int off = 32; off > 0; off >>= 1) loss += __shfl_xor(loss, off);
    if (lane == 0) sRed[t >> 6] = loss;
    __syncthreads();
    if (t < rows) partials[(size_t)blockIdx.x * rows + t] = t == 0 ? (sRed[0] + sRed[1]) + (sRed[2] + sRed[3]) : 0.0;
    return;
  }
  if (!do_acc) return;
  if (rows == 1 && G2 > 1) {  // the G2 groups' sums folded in LDS (fixed order): one row per workgroup
    __syncthreads();          // every thread is done with the tile's LDS
    double* sF = reinterpret_cast<double*>(smem);  // [G2][2k][F]
    if (g2 < G2 && fb < F)
#pragma unroll
      for (int j = 0; j < KP; ++j)
        if (j < k) {
          sF[(g2 * 2 * k + j) * F + fb] = A64[0][j];
          sF[(g2 * 2 * k + k + j) * F + fb] = D64[0][j];
        }
    __syncthreads();
    double* prow = partials + (size_t)blockIdx.x * (2 * k * F);
    for (int e = t; e < 2 * k * F; e += NT) {
      double v = 0.0;
      for (int g = 0; g < G2; ++g) v += sF[(size_t)g * 2 * k * F + e];
      prow[e] = v;
    }
    return;
  }
  if (g2 >= G2) return;
  double* prow = partials + ((size_t)blockIdx.x * G2 + g2) * (2 * k * F);
#pragma unroll
  for (int u = 0; u < NFT; ++u) {
    const int f = fb + NT * u;
    if (f < F)
#pragma unroll
      for (int j = 0; j < KP; ++j)
        if (j < k) {
          prow[j * F + f] = A64[u][j];
          prow[k * F + j * F + f] = D64[u][j];
        }
  }
}

// H <- H ∘ A / D (D == 0 -> EPS32, SK:706), AD = [A | D] reduced over all samples (and ranks)
__global__ __launch_bounds__(256) void wmu_basis_kernel(const double* __restrict__ AD, double* __restrict__ H64, int kF) {
  for (int e = blockIdx.x * 256 + threadIdx.x; e < kF; e += gridDim.x * 256) {
    double d = AD[kF + e];
    if (d == 0.0) d = EPS32;
    H64[e] = H64[e] * (AD[e] / d);
  }
}

// ------------------------------------------------------------------------------------------------
// wmu_iter_wt_kernel — n weighted MU iterations as ONE persistent launch (fp32 X and M, F = 81,
// k = 4, W resident in LDS).  The layout is mu_iter_wt_kernel's (§3.0 of DESIGN.md): one 4-wave
// workgroup per CU, each wave on its own 16-sample tiles (the same tiles every iteration), no
// barrier inside an iteration, the next tiles' X AND M prefetched into AGPRs by counted loads, the
// workgroup's fp64 row reduced in-launch by the ticket tree, every workgroup applying the H-step
// itself.  Lane l = 4s + e of a tile: sample s, features [21e, 21e + 21) (the lanes past F read
// zero-Hᵀ pads).  Per tile (the arithmetic of wmu_pass_kernel, oracle/wmu_ref.py):
//   phase 1  rec_f = w·h_f, mx_f = m_f·x_f, mr_f = m_f·rec_f; num_j = Σ_f mx_f·h_jf and
//            den_j = Σ_f mr_f·h_jf over the lane's features in packed fp32 chains of 7 folded into
//            fp64, then the fp64 reduce-scatter over the sample's 4 lanes: lane e owns (num_e,
//            den_e); w'_e = w_e·num_e/den_e (den = 0 -> EPS32)
//   phase 3  rec'_f = w'·h_f; A_jf += w'_j·mx_f, D_jf += w'_j·m_f·rec'_f (fp32 per lane over the
//            iteration's tiles)
// End of an iteration: each lane class's sums over the wave's 16 sample lanes, the 4 waves in wave
// order in fp64 -> the workgroup's row [A | D] (2kF = 648 doubles), the ticket tree -> AD, and
// H <- H∘A/D (D = 0 -> EPS32) in every workgroup.  Deterministic: no order depends on arrival.
// ------------------------------------------------------------------------------------------------
namespace ww {
using G4 = wt::Geo<4>;
constexpr int K = 4, NL = 4, TSW = 16, F = wt::F, NQ = G4::NQ, KF = K * F;
constexpr int NOUT = 2 * KF;             // [A | D]
constexpr int NACC = 2 * NQ * K;         // fp32 accumulators per lane: A then D
constexpr int L_STG = 0;                 // [NWV][2][XSTR]: the wave's X slot, then its M slot
constexpr int L_RED = L_STG + wt::NWV * 2 * G4::XSTR;          // [NWV][NL][NACC] fp32
constexpr int L_H = L_RED + wt::NWV * NL * NACC * 4;           // H fp64 [K][F]
constexpr int L_AB = L_H + KF * 8;                             // AD fp64 [NOUT]
constexpr int L_HT = L_AB + NOUT * 8;                          // Hᵀ fp32 [NL·NQ][K]
constexpr int L_FLAG = L_HT + NL * NQ * K * 4;                 // 4 ints
constexpr int L_WRES = (L_FLAG + 16 + 15) / 16 * 16;           // [NWV][nbt_max][WBW]
static_assert(L_RED % 16 == 0 && L_HT % 16 == 0, "16-byte aligned LDS regions");
static_assert(NOUT <= 3 * NT, "three accumulator outputs per thread at most");
}  // namespace ww

struct WmuPersistArgs {
  const float* X;
  const float* M;
  float* W;
  double* H64;       // in: the basis; out: the final basis
  double* partials;  // [G][NOUT] per-workgroup rows
  double* groups;    // [NG][NOUT] group rows
  double* AD;        // [NOUT]: out (the last iteration's reduced accumulators)
  uint32_t* cnt;     // CNT_WORDS counters (at rest on entry, left at rest)
  int64_t n_tiles;
  int n_iter;
  int n_groups;
  uint64_t* xctl;    // MULTI: the cross-rank exchange control block (mu_iter_wt_kernel's protocol)
};

// Hᵀ (fp32, the lanes' feature blocks, rows >= F zero) from the fp64 H in LDS
__device__ __forceinline__ void ww_derive_basis(unsigned char* smem, int t) {
  const double* sH = reinterpret_cast<const double*>(smem + ww::L_H);
  float* sHt = reinterpret_cast<float*>(smem + ww::L_HT);
  for (int e = t; e < ww::NL * ww::NQ * ww::K; e += NT) {
    const int f = e / ww::K;
    const int j = e - f * ww::K;
    sHt[e] = f < ww::F ? (float)sH[j * ww::F + f] : 0.f;
  }
  __syncthreads();
}
// H <- H ∘ A / D from AD in LDS (D = 0 -> EPS32; oracle/wmu_ref.update_h), then Hᵀ
__device__ __forceinline__ void ww_update_basis(unsigned char* smem, int t) {
  constexpr int U = (ww::KF + NT - 1) / NT;
  double* sH = reinterpret_cast<double*>(smem + ww::L_H);
  const double* sAD = reinterpret_cast<const double*>(smem + ww::L_AB);
  double hn[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = t + NT * u;
    hn[u] = 0.0;
    if (e < ww::KF) {
      double d = sAD[ww::KF + e];
      if (d == 0.0) d = EPS32;
      hn[u] = sH[e] * (sAD[e] / d);
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (t + NT * u < ww::KF) sH[t + NT * u] = hn[u];
  __syncthreads();
  ww_derive_basis(smem, t);
}

namespace cnmf::wt {
template <int N>
__device__ __forceinline__ void wait_set12(u32x4 (&pf)[12]) {
  asm volatile("s_waitcnt vmcnt(%12)"
               : "+a"(pf[0]), "+a"(pf[1]), "+a"(pf[2]), "+a"(pf[3]), "+a"(pf[4]), "+a"(pf[5]), "+a"(pf[6]),
                 "+a"(pf[7]), "+a"(pf[8]), "+a"(pf[9]), "+a"(pf[10]), "+a"(pf[11])
               : "n"(N) : "memory");
}
}  // namespace cnmf::wt

template <int PD, bool MULTI = false>
__global__ __launch_bounds__(NT, 1) void wmu_iter_wt_kernel(WmuPersistArgs a) {
  using namespace wt;
  using G4 = Geo<4>;
  constexpr int KK = ww::K, NL = ww::NL, TSW = ww::TSW, NQ = ww::NQ, NOUT = ww::NOUT, NACC = ww::NACC;
  constexpr int KF = ww::KF;
  constexpr int XBW = G4::XBW, XSTR = G4::XSTR, WBW = G4::WBW, PFW = G4::PFW, LASTL = G4::LASTL;
  constexpr int PFS = 2 * PFW;  // loads per prefetch set: the X tile, then the M tile
  static_assert(PFS == 12, "wait_set12");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int t = threadIdx.x;
  const int l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int s = l / NL, e = l % NL;
  const int b = blockIdx.x;
  const int G = gridDim.x;
  const int NW = NWV * G;
  const int gw = NWV * b + w;
  const int NG = a.n_groups;
  const int g = b % NG;
  const int gs = (G - g + NG - 1) / NG;
  const unsigned char* Xb = reinterpret_cast<const unsigned char*>(a.X);
  const unsigned char* Mb = reinterpret_cast<const unsigned char*>(a.M);
  unsigned char* Wb = reinterpret_cast<unsigned char*>(a.W);
  const int nbt = (int)((a.n_tiles - gw + NW - 1) / NW);  // this wave's tiles per iteration
  const int nbt_max = (int)((a.n_tiles + NW - 1) / NW);
  unsigned char* stx = smem + ww::L_STG + 2 * w * XSTR;
  unsigned char* stm = stx + XSTR;
  float* wres = reinterpret_cast<float*>(smem + ww::L_WRES + (size_t)w * nbt_max * WBW);  // [i][TSW][K]
  float* red = reinterpret_cast<float*>(smem + ww::L_RED);
  double* sH = reinterpret_cast<double*>(smem + ww::L_H);
  double* sAD = reinterpret_cast<double*>(smem + ww::L_AB);
  int* sFlag = reinterpret_cast<int*>(smem + ww::L_FLAG);
  uint32_t* cnt_group = a.cnt + CNT_GROUP0 + 32 * g;
  uint32_t* cnt_top = a.cnt + CNT_TOP;
  uint32_t* flag = a.cnt + CNT_FLAG;
  uint32_t* err = a.cnt + CNT_ERR;

  // ---- the basis, the staging pads (finite zeros past both slots), this wave's W tiles
  for (int i = t; i < KF; i += NT) sH[i] = a.H64[i];
  if (l < G4::PADB / 4) {
    reinterpret_cast<float*>(stx + XBW)[l] = 0.f;
    reinterpret_cast<float*>(stm + XBW)[l] = 0.f;
  }
  for (int c = l; c < nbt * (WBW / 16); c += 64) {
    const int i = c / (WBW / 16), ch = c - i * (WBW / 16);
    *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned char*>(wres) + i * WBW + 16 * ch) =
        *reinterpret_cast<const u32x4*>(Wb + (size_t)(gw + (int64_t)NW * i) * WBW + 16 * ch);
  }
  __syncthreads();
  ww_derive_basis(smem, t);

  // the lane's Hᵀ: fp32 component pairs of each of its NQ features
  f2 hp[NQ][2];
  auto load_basis = [&]() {
    const float* sHt = reinterpret_cast<const float*>(smem + ww::L_HT);
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      const float4 h = *reinterpret_cast<const float4*>(sHt + (NQ * e + c) * KK);
      hp[c][0] = f2{h.x, h.y};
      hp[c][1] = f2{h.z, h.w};
    }
  };
  load_basis();

  f2 accA[NQ][2], accD[NQ][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int c = 0; c < NQ; ++c)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        accA[c][q] = f2{0.f, 0.f};
        accD[c][q] = f2{0.f, 0.f};
      }
  };
  zero_acc();

  // the tile's 16-byte chunks of this lane in X, then the same chunks of M (lanes >= LASTL re-load
  // chunk l for the last load: never staged; every lane issues the same loads)
  auto prefetch = [&](u32x4 (&pf)[PFS], int64_t tile) {
    const size_t off = (size_t)tile * XBW + 16 * l;
#pragma unroll
    for (int u = 0; u < PFW - 1; ++u) ld16(pf[u], Xb + off + 1024 * u);
    ld16(pf[PFW - 1], Xb + (l < LASTL ? off + 1024 * (PFW - 1) : off));
#pragma unroll
    for (int u = 0; u < PFW - 1; ++u) ld16(pf[PFW + u], Mb + off + 1024 * u);
    ld16(pf[2 * PFW - 1], Mb + (l < LASTL ? off + 1024 * (PFW - 1) : off));
  };
  auto stage = [&](const u32x4 (&pf)[PFS]) {
    const unsigned ax = (unsigned)(uintptr_t)(stx + 16 * l);
    const unsigned am = (unsigned)(uintptr_t)(stm + 16 * l);
    stage_rec<0, PFW - 1>(ax, pf);
    if (l < LASTL) st16<1024 * (PFW - 1)>(ax, pf[PFW - 1]);
    stage_rec<0, PFW - 1>(am, pf + PFW);
    if (l < LASTL) st16<1024 * (PFW - 1)>(am, pf[2 * PFW - 1]);
  };

  const int total = a.n_iter * nbt;
  u32x4 pf[PD][PFS];
#pragma unroll
  for (int k = 0; k < PD; ++k) prefetch(pf[k], gw + (int64_t)NW * k);  // the host keeps nbt > PD
  TL_START;

  bool alive = true;
  int cur_i = 0, cur_it = 0, nx_i = PD;
  auto step = [&](u32x4 (&pfk)[PFS]) {
    wait_set12<PFS * (PD - 1)>(pfk);  // the PD - 1 younger sets stay in flight
    stage(pfk);
    prefetch(pfk, gw + (int64_t)NW * nx_i);
    if (++nx_i == nbt) nx_i = 0;
  };
  auto body = [&]() {
    const int it = cur_it, i = cur_i;
    if (++cur_i == nbt) {
      cur_i = 0;
      ++cur_it;
    }
    const bool last_it = it + 1 == a.n_iter;
    // phase 1
    const float* xr = reinterpret_cast<const float*>(stx) + s * wt::F + NQ * e;
    const float* mr = reinterpret_cast<const float*>(stm) + s * wt::F + NQ * e;
    float mv[NQ], mx[NQ];
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      mv[c] = mr[c];
      mx[c] = mv[c] * xr[c];
    }
    float* wt_ = wres + i * (TSW * KK);
    const float4 w4 = *reinterpret_cast<const float4*>(wt_ + s * KK);
    const f2 w01 = f2{w4.x, w4.y}, w23 = f2{w4.z, w4.w};
    const double wold = (double)(e == 0 ? w4.x : (e == 1 ? w4.y : (e == 2 ? w4.z : w4.w)));
    double pn[KK], pd[KK];
#pragma unroll
    for (int c0 = 0; c0 < NQ; c0 += 7) {
      f2 cn[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}}, cd[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
      for (int c = c0; c < c0 + 7; ++c) {
        f2 r2 = w01 * hp[c][0];
        r2 = __builtin_elementwise_fma(w23, hp[c][1], r2);
        const float mrc = mv[c] * (r2.x + r2.y);
        const f2 xx = f2{mx[c], mx[c]}, rr = f2{mrc, mrc};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          cn[q] = __builtin_elementwise_fma(xx, hp[c][q], cn[q]);
          cd[q] = __builtin_elementwise_fma(rr, hp[c][q], cd[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (c0 == 0) {
          pn[2 * q] = (double)cn[q].x;
          pn[2 * q + 1] = (double)cn[q].y;
          pd[2 * q] = (double)cd[q].x;
          pd[2 * q + 1] = (double)cd[q].y;
        } else {
          pn[2 * q] += (double)cn[q].x;
          pn[2 * q + 1] += (double)cn[q].y;
          pd[2 * q] += (double)cd[q].x;
          pd[2 * q + 1] += (double)cd[q].y;
        }
      }
    }
    // reduce-scatter over the sample's 4 lanes (fp64): lane e keeps component e
    const bool b1 = (e & 1) != 0, b2 = (e & 2) != 0;
    double kn[2], kd[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const double keepn = b2 ? pn[2 + m] : pn[m], sendn = b2 ? pn[m] : pn[2 + m];
      const double keepd = b2 ? pd[2 + m] : pd[m], sendd = b2 ? pd[m] : pd[2 + m];
      kn[m] = keepn + dpp64<0x4E>(sendn);  // quad_perm [2,3,0,1]
      kd[m] = keepd + dpp64<0x4E>(sendd);
    }
    const double num = (b1 ? kn[1] : kn[0]) + dpp64<0xB1>(b1 ? kn[0] : kn[1]);  // quad_perm [1,0,3,2]
    double den = (b1 ? kd[1] : kd[0]) + dpp64<0xB1>(b1 ? kd[0] : kd[1]);
    if (den == 0.0) den = EPS32;
    const float wn = (float)(wold * div_nr(num, den));
    wt_[s * KK + e] = wn;
    // phase 3 with the sample's new row (this wave's writes above precede the read)
    const float4 p4 = *reinterpret_cast<const float4*>(wt_ + s * KK);
    const f2 wp[2] = {f2{p4.x, p4.y}, f2{p4.z, p4.w}};
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      f2 r2 = wp[0] * hp[c][0];
      r2 = __builtin_elementwise_fma(wp[1], hp[c][1], r2);
      const float mrc = mv[c] * (r2.x + r2.y);
      const f2 xx = f2{mx[c], mx[c]}, rr = f2{mrc, mrc};
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        accA[c][q] = __builtin_elementwise_fma(xx, wp[q], accA[c][q]);
        accD[c][q] = __builtin_elementwise_fma(rr, wp[q], accD[c][q]);
      }
    }
    if (i + 1 != nbt) return;

    // ---- end of this wave's iteration: its sums over the sample lanes of each e -> LDS
    // (the all-reduce form: mu_iter_wt_kernel's reduce-scatter spills this kernel past 512 registers)
    {
      float* rw = red + (w * NL + e) * NACC;
#pragma unroll
      for (int c = 0; c < NQ; ++c) {
        const float4 va = make_float4(sum_over_samples<NL>(accA[c][0].x), sum_over_samples<NL>(accA[c][0].y),
                                      sum_over_samples<NL>(accA[c][1].x), sum_over_samples<NL>(accA[c][1].y));
        const float4 vd = make_float4(sum_over_samples<NL>(accD[c][0].x), sum_over_samples<NL>(accD[c][0].y),
                                      sum_over_samples<NL>(accD[c][1].x), sum_over_samples<NL>(accD[c][1].y));
        if (l < NL) {
          *reinterpret_cast<float4*>(rw + c * KK) = va;
          *reinterpret_cast<float4*>(rw + NQ * KK + c * KK) = vd;
        }
      }
    }
    zero_acc();
    __syncthreads();
    // the workgroup's fp64 row [A | D]: the four waves' sums in wave order (deterministic)
    {
      double* prow = a.partials + (size_t)b * NOUT;
      auto row_val = [&](int o) {
        const int isd = o >= KF ? 1 : 0;
        const int r = o - isd * KF;
        const int j = r / wt::F;
        const int f = r - j * wt::F;
        const int ee = f / NQ;
        const float* rr = red + ee * NACC + isd * NQ * KK + (f - NQ * ee) * KK + j;
        constexpr int WS = NL * NACC;  // wave stride
        return ((double)rr[0] + (double)rr[WS]) + ((double)rr[2 * WS] + (double)rr[3 * WS]);
      };
      // pairs of doubles, one 16-byte sc1 store each (round 6: the tree's hand-offs in 16-byte chunks)
      static_assert(NOUT % 2 == 0, "[A | D] rows are whole 16-byte chunks");
      if constexpr (MULTI) {  // (the multi-GPU form keeps the round-5 hand-offs throughout)
        for (int o = t; o < NOUT; o += NT) __hip_atomic_store(prow + o, row_val(o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        for (int c = t; c < NOUT / 2; c += NT) st16_sc1v(prow + 2 * c, row_val(2 * c), row_val(2 * c + 1));
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores landed
    __syncthreads();
    TL(it, 0);
    if (t == 0) {
      const uint32_t old = __hip_atomic_fetch_add(cnt_group, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sFlag[0] = old == (uint32_t)((it + 1) * gs - 1);
      sFlag[1] = 0;
      sFlag[2] = 1;
    }
    __syncthreads();
    if (sFlag[0]) {  // group combiner
      // (the MULTI form keeps the 8-byte sum: at 512 registers the 16-byte batches spilled)
      if constexpr (MULTI) sum_rows_n<NOUT>(a.partials, g, NG, gs, nullptr, a.groups + (size_t)g * NOUT, t);
      else sum_rows_v<NOUT>(a.partials, g, NG, gs, nullptr, a.groups + (size_t)g * NOUT, t);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) {
        const uint32_t old = __hip_atomic_fetch_add(cnt_top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sFlag[1] = old == (uint32_t)((it + 1) * NG - 1);
      }
      __syncthreads();
      if (sFlag[1]) {  // top combiner: AD
        if constexpr (MULTI) {
          sum_rows_n<NOUT>(a.groups, 0, 1, NG, sAD, a.AD, t);
          xchg_allreduce_n<NOUT>(a.xctl, a.AD, sAD, err, it, t);  // + the other ranks' [A|D]
        } else {
          sum_rows_v<NOUT>(a.groups, 0, 1, NG, sAD, a.AD, t);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0 && !last_it)
          __hip_atomic_store(flag, (uint32_t)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        TL_PUB(it);
      }
    }
    const bool top = sFlag[1] != 0;
    if (last_it) {
      alive = false;
      for (int c = l; c < nbt * (WBW / 16); c += 64) {  // this wave's W back to HBM, once per launch
        const int ii = c / (WBW / 16), ch = c - ii * (WBW / 16);
        *reinterpret_cast<u32x4*>(Wb + (size_t)(gw + (int64_t)NW * ii) * WBW + 16 * ch) =
            *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(wres) + ii * WBW + 16 * ch);
      }
      if (!top) return;
      // the last combiner of the launch: every other workgroup has arrived for the last time
      ww_update_basis(smem, t);
      for (int o = t; o < KF; o += NT) a.H64[o] = sH[o];
      if (t < NG) __hip_atomic_store(a.cnt + CNT_GROUP0 + 32 * t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == 0) {
        __hip_atomic_store(cnt_top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (MULTI)  // the next launch's generations follow this one's
          __hip_atomic_fetch_add(a.xctl + XC_GEN, (uint64_t)a.n_iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (!top) {
      if (t == 0) {
        const uint32_t want = (uint32_t)(it + 1);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (true) {  // the flag and the error word in one batch: one round trip per round
          const uint32_t ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) break;
          if (ev != 0u) {
            sFlag[2] = 0;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > sl::SPIN_TIMEOUT) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sFlag[2] = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      if (!sFlag[2]) {  // a workgroup never arrived (not co-resident): give up, error word set
        alive = false;
        return;
      }
      if constexpr (MULTI) {
        for (int o = t; o < NOUT; o += NT) sAD[o] = ld_sc1(a.AD + o);
      } else {  // 16-byte sc1 loads, all in flight together (round 6)
        constexpr int NCH = NOUT / 2;
        const int c0 = t < NCH ? t : 0, c1 = t + NT < NCH ? t + NT : 0;
        u32x4 r0, r1;
        ld16_sc1(r0, a.AD + 2 * c0);
        if (NCH > NT) ld16_sc1(r1, a.AD + 2 * c1);
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(r0), "+v"(r1) : : "memory");
        if (t < NCH) {
          sAD[2 * t] = lo_d(r0);
          sAD[2 * t + 1] = hi_d(r0);
        }
        if (t + NT < NCH) {
          sAD[2 * (t + NT)] = lo_d(r1);
          sAD[2 * (t + NT) + 1] = hi_d(r1);
        }
      }
      __syncthreads();
    }
    ww_update_basis(smem, t);
    load_basis();
    TL(it, 1);
  };

  for (int p = 0; p < total && alive; p += PD) {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      step(pf[k]);
      if (p + k < total && alive) body();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
}

// ------------------------------------------------------------------------------------------------
// als_iter_wt_kernel — n constrained-ALS iterations (§8 a7, cfg5; spec oracle/als_ref.py) as ONE
// persistent launch (fp32 X, F = 81, k = 4).  The wave-tile layout of mu_iter_wt_kernel (one 4-wave
// workgroup per CU, each wave on its own 16-sample tiles, the next tiles' X prefetched into AGPRs by
// counted loads), with the W-step of als_pass_sl_kernel and the H-step of als_basis_kernel:
//   phase 1  c = H·x + δ² in fp64: lane (s, e) forms its 21 features' partials from the fp64 Hᵀ in
//            LDS; a quad butterfly sums them ((p0 + p1) + (p2 + p3): every lane the same bits, and
//            the same bits as als_pass_sl_kernel's four feature blocks)
//   FCLS     lane e evaluates the passive sets e, e + 4, e + 8, e + 12 from the table in LDS; the
//            least objective among the feasible (ties: lowest mask) by quad shuffles;
//            w_e = max(T_best·c, 0).  The W-step is exact (it never reads the old W), so W is only
//            written, once per tile, 256 contiguous bytes per wave
//   phase 3  A += w'ᵀx, B += w'ᵀw' in fp32 per lane over the iteration (mu_iter_wt_kernel's)
// End of an iteration: the workgroup's fp64 row [WᵀX | WᵀW], the ticket tree -> AB, and in EVERY
// workgroup the H-step sweep (als_hstep: deterministic, so every workgroup holds the same bits),
// then Hᵀ, HHᵀ and the next W-step's table — no broadcast of the new basis.
// ------------------------------------------------------------------------------------------------
namespace wa {
using G4 = wt::Geo<4>;
constexpr int K = 4, NL = 4, TSW = 16, F = wt::F, NQ = G4::NQ, V = F + K, NOUT = K * V;
constexpr int NACC = G4::NACC;                                  // NQ·K + K fp32 accumulators
constexpr int L_STG = 0;                                        // [NWV][XSTR]
constexpr int L_RED = L_STG + wt::NWV * G4::XSTR;               // [NWV][NL][NACC] fp32
constexpr int L_AB = L_RED + wt::NWV * NL * NACC * 4;           // AB fp64 [K][V] (the top's sum; TOL: + loss)
constexpr int L_HT = L_AB + (NOUT + 2) * 8;                     // Hᵀ fp64 [NL·NQ][K], rows >= F zero
constexpr int L_HHT = L_HT + NL * NQ * K * 8;                   // HHᵀ fp64 [K][K]
// passive-set table, masks at a stride of TSTR doubles (18: the four masks a quad reads with one
// ds_read_b128 land on disjoint banks; at 16 the masks e and e + 2 shared them), then 16 flags
constexpr int TSTR = 18;
constexpr int L_TAB = L_HHT + K * K * 8;
constexpr int L_FLAG = L_TAB + (16 * TSTR + 16) * 8;            // 4 ints
constexpr int L_LOSS = (L_FLAG + 16 + 15) / 16 * 16;            // TOL: [NWV] wave loss sums, init, prev
constexpr int L_WSTG = L_LOSS + 8 * 8;                          // TOL: [NWV] the old W tile (256 B)
constexpr int L_LACC = L_WSTG + wt::NWV * 256;                  // TOL: [NWV][64] the lanes' loss sums
constexpr int L_HS = L_LACC + wt::NWV * 64 * 8;                 // als_hstep's arrays (als_lds_bytes)
constexpr int L_H = L_HS + K * F * 8;                           // H fp64 [K][F]: the H-step's own sH
static_assert(L_RED % 16 == 0 && L_HT % 16 == 0 && L_HS % 16 == 0, "16-byte aligned LDS regions");
static_assert(NOUT * 8 >= wt::NWV * 64 * 4, "the prologue's dummy stores stay inside the partial row");
}  // namespace wa

struct AlsPersistArgs {
  const float* X;
  float* W;
  double* H64;       // in: the basis; out: the final basis
  double* Ht;        // out [F][4] fp64
  double* HHt;       // out [4][4]
  double* table;     // out: the next W-step's table
  double* partials;  // [G][K*V]
  double* groups;    // [NG][K*V]
  double* AB;        // [K*V] out: the last iteration's reduced accumulators
  uint32_t* cnt;     // CNT_WORDS counters (at rest on entry, left at rest)
  int64_t n_tiles;
  int n_iter;
  int n_groups;
  double delta2;     // sum_to_one²
  double lam;        // smoothness
  uint64_t* xctl;    // MULTI: the cross-rank exchange control block (mu_iter_wt_kernel's protocol)
  int prio;          // the issue-priority ladder's band (steps; 0 = off)
  double* tolctl;    // TOL: the tolerance-test control block (cnmf_mu_fit_tol's layout)
};

// Hᵀ (fp64, the lanes' feature blocks), HHᵀ (fp64; 16 threads per entry, fixed xor tree) and the
// passive-set table, from the fp64 H in LDS
__device__ __forceinline__ void wa_derive(unsigned char* smem, int t, double delta2) {
  using namespace wa;
  const double* sH = reinterpret_cast<const double*>(smem + L_H);
  double* sHt = reinterpret_cast<double*>(smem + L_HT);
  double* sHHt = reinterpret_cast<double*>(smem + L_HHT);
  for (int e = t; e < NL * NQ * K; e += NT) {
    const int f = e / K;
    const int j = e - f * K;
    sHt[e] = f < F ? sH[j * F + f] : 0.0;
  }
  constexpr int TPE = NT / (K * K);
  const int en = t / TPE, part = t - en * TPE;
  const int j = en / K, m = en - (en / K) * K;
  double v = 0.0;
  for (int f = part; f < F; f += TPE) v = fma(sH[j * F + f], sH[m * F + f], v);
#pragma unroll
  for (int o = TPE / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (part == 0) sHHt[en] = v;
  __syncthreads();
  PH(8);
  als_table(sHHt, K, K, delta2, reinterpret_cast<double*>(smem + L_TAB), t, TSTR);
  __syncthreads();
}

// The H-step: AB is in the H-step's A / B arrays already (the workgroups that load it scatter it
// there; copy_ab: the top combiner's sum, from sAB) and H is the H-step's own sH (no copies in or
// out: 0.4 + 0.3 µs).  One Gauss-Seidel sweep of exact NNLS rows (als_hstep), then wa_derive
// (inlined once, after the kernel's streaming loop)
__device__ __forceinline__ void wa_update_basis(int t, double lam, double delta2, bool copy_ab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  using namespace wa;
  const double* sAB = reinterpret_cast<const double*>(smem + L_AB);
  double* hA = reinterpret_cast<double*>(smem + L_HS);
  double* hB = hA + 2 * K * F;
  if (copy_ab) {
    for (int e = t; e < K * F; e += NT) hA[e] = sAB[(e / F) * V + (e % F)];
    if (t < K * K) hB[t] = sAB[(t / K) * V + F + (t % K)];
  }
  __syncthreads();
  PH(2);
#ifdef CNMF_ALS_NOHSTEP  // timing-only diagnostic: the persistent ALS without its H-step rows (H fixed)
  __syncthreads();
#else
  als_hstep(smem + L_HS, F, K, lam, t);
#endif
  PH(5);
  wa_derive(smem, t, delta2);
  PH(6);
}

// HREG (diagnostic A/B, one workgroup per CU): the lane's fp64 Hᵀ rows held in VGPRs for the
// iteration instead of re-read from LDS every tile (42 ds_read_b128 per wave tile).
// MF: phase 1 (c = H·x, fp64) on the matrix cores — 21 v_mfma_f64_4x4x4f64 per wave tile instead of
// 84 fp64 FMAs, 42 ds_read_b128 of Hᵀ and the quad butterfly.  The instruction's operand layout
// (profiles/r04/mfma_f64_layout.txt): A[b][i][k] at lane i + 4b + 16k, B[b][k][j] at lane
// j + 4b + 16k, D[b][i][j] at lane 16i + 4b + j.  So with sample s = 4i + b the result c[s][j] lands
// on lane 4s + j (the FCLS's quad layout) when lane L holds x of sample 4(L % 4) + (L / 4) % 4 and
// feature group k = L / 16 (features 21k .. 21k + 20; B = H[j][21k + q] from VGPRs); phase 3 then
// takes the sample's new row w' through the wave's LDS slot and its sums run over the 16 lanes of a
// row (one feature group).  MFL: the B operand read from LDS per tile (ds_read_b64) instead of VGPRs.
// MX: the whole W-step on the matrix cores (fp64), lane l = (sample s = l % 16, residue g = l / 16):
//   phase 1  c[q][s] = Σ_f H[q][f]·x[s][f] on 21 v_mfma_f64_4x4x4f64 with A = H[q = l % 4][4ks + g]
//            and B = x[s][4ks + g] (the lane's features are f ≡ g mod 4), so D lands on lane 16q + s:
//            lane (s, g) holds c[g][s] — exactly the B operand of
//   FCLS     four v_mfma_f64_16x16x4f64 (K = the 4 components): block b' evaluates the masks 4b' + i % 4
//            for all 16 samples, A row i = (mask 4b' + i % 4, component r = (i / 4) ^ (i % 4)) of the
//            table; the f64 16x16 D layout (row g + 4·reg on lane s + 16g) leaves on lane (s, g) the
//            whole solution vector of mask 4b' + g, rotated: register ρ = component ρ ^ g.  With c
//            rotated the same way (c[g ^ ρ] from lanes l ^ 16ρ by permlane swaps) the objective
//            −½ c·v, the feasibility test and the choice (least objective, ties the lowest mask) are
//            per-lane register work plus two swap rounds; w[s][g] = max(T_best[g]·c, 0) from the table.
//   phase 3  A[g ^ ρ][4ks + g] += x·w[s][g ^ ρ], B[g][g ^ ρ] += w[s][g]·w[s][g ^ ρ] (rotated, fp32 per
//            lane); the end of the iteration sums the 16 lanes of a row and un-rotates into the
//            reduction's layout.
//
// TOL (MX only; cnmf_als_fit_tol): the tolerance test of oracle/als_ref.py (SK:872-884's rule) on the
// device, as mu_iter_wt_kernel's: in iteration g + 1 (g % 10 == 0) every lane also accumulates
// ‖x − w·H‖² of the state after g iterations — x and H_g are the pass's, W_g is the tile's W read
// with X (every TOL step prefetches it: the W-step itself never reads W) — carried as one more
// column of the partial rows; the top combiner applies the test, and on a stop every workgroup leaves
// with H_g (this iteration's H-step not applied) while the loss iterations' copies of W_g in the
// snapshot buffer give the host W_g.
template <int PD, int OCC, bool MULTI = false, bool HREG = false, bool MF = false, bool MFL = false, bool MX = false,
          bool TOL = false>
__global__ __launch_bounds__(NT, OCC) void als_iter_wt_kernel(AlsPersistArgs a) {
  using namespace wt;
  using G4 = Geo<4>;
  static_assert(!TOL || MX, "the device tolerance test is the MX kernel's");
  constexpr int KK = wa::K, NL = wa::NL, NQ = wa::NQ, V = wa::V, NOUT = wa::NOUT, NACC = wa::NACC;
  constexpr int NOUTT = NOUT + (TOL ? 1 : 0);  // partial-row width: + the loss of the checked state
  // round 6: the reduction tree's hand-offs as 16-byte sc1 loads / stores where the rows are whole
  // chunks (NOUTT even: not the TOL form, whose rows keep cnmf_als_fit_tol's k(F+k) + 1)
  constexpr bool VT = NOUTT % 2 == 0;
  static_assert(!VT || NOUTT / 2 <= NT, "one 16-byte chunk of a row per thread");
  constexpr int XBW = G4::XBW, XSTR = G4::XSTR, PFW = G4::PFW, LASTL = G4::LASTL;
  // MX: the W-step starts from the passive set of the tile's previous W (WARM, round 5), so its W is
  // loaded with X, as the TOL form's loss needs it too
  constexpr bool WARM = MX;
  constexpr int PFS = PFW + (TOL || WARM ? 1 : 0);  // loads per prefetch set: the X tile (+ its old W)
  constexpr int KP = KK / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int t = threadIdx.x;
  const int l = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int s = l / NL, e = l % NL;
  // the sample and feature group whose x this lane holds (phases 1 and 3): MF the matrix-core A layout
  const int sx = MF ? 4 * (l & 3) + ((l >> 2) & 3) : s, ex = MF ? (l >> 4) : e;
  const int b = blockIdx.x;
  const int G = gridDim.x;
  const int NW = NWV * G;
  const int gw = NWV * b + w;
  const int NG = a.n_groups;
  const int g = b % NG;
  const int gs = (G - g + NG - 1) / NG;
  const unsigned char* Xb = reinterpret_cast<const unsigned char*>(a.X);
  const int nbt = (int)((a.n_tiles - gw + NW - 1) / NW);  // this wave's tiles per iteration
  unsigned char* stg = smem + wa::L_STG + w * XSTR;
  float* red = reinterpret_cast<float*>(smem + wa::L_RED);
  double* sH = reinterpret_cast<double*>(smem + wa::L_H);
  double* sAB = reinterpret_cast<double*>(smem + wa::L_AB);
  const double* sHtl = reinterpret_cast<const double*>(smem + wa::L_HT) + NQ * e * KK;
  const double* sTab = reinterpret_cast<const double*>(smem + wa::L_TAB);
  int* sFlag = reinterpret_cast<int*>(smem + wa::L_FLAG);
  uint32_t* cnt_group = a.cnt + CNT_GROUP0 + 32 * g;
  uint32_t* cnt_top = a.cnt + CNT_TOP;
  uint32_t* flag = a.cnt + CNT_FLAG;
  uint32_t* err = a.cnt + CNT_ERR;
  // TOL: the launch's first global iteration, the test's error at init and previous error (every
  // workgroup tracks them itself), the snapshot buffer of W_g, the wave's old-W staging
  // (uniform values in SGPRs, and each lane's loss sum in LDS: no long-lived VGPR in the streaming
  // loop, whose spill reloads would wait on — drain — the prefetch)
  const int it0 = TOL ? __builtin_amdgcn_readfirstlane((int)ld_sc1(a.tolctl + TC_IT0)) : 0;
  const double tolv = TOL ? ld_sc1(a.tolctl + TC_TOL) : 0.0;
  double* sLoss = reinterpret_cast<double*>(smem + wa::L_LOSS);
  double* lacc = reinterpret_cast<double*>(smem + wa::L_LACC) + 64 * w + l;
  if (TOL) *lacc = 0.0;
  if (TOL && t == 0) {
    sLoss[4] = ld_sc1(a.tolctl + TC_INIT);
    sLoss[5] = ld_sc1(a.tolctl + TC_PREV);
    sLoss[6] = tolv;  // the test reads it from LDS (a register across the loop was spilled)
  }
  float* wsnap = nullptr;
  if (TOL) {
    const long long wp = __double_as_longlong(ld_sc1(a.tolctl + TC_WSNAP));
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(wp & 0xFFFFFFFFll));
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(wp >> 32));
    wsnap = reinterpret_cast<float*>(((unsigned long long)hi << 32) | lo);
  }
  unsigned char* wstg = smem + wa::L_WSTG + w * 256;
  unsigned char* Wb = reinterpret_cast<unsigned char*>(a.W);
  int cur_it = 0;  // the iteration the streaming loop is in

  // ---- the basis for the first iteration, Hᵀ / HHᵀ / table, the staging pad
  for (int i = t; i < KK * wa::F; i += NT) sH[i] = a.H64[i];
  if (l < G4::PADB / 4) reinterpret_cast<float*>(stg + XBW)[l] = 0.f;
  __syncthreads();
  wa_derive(smem, t, a.delta2);
  double hreg[HREG ? NQ : 1][KK];
  double hb[MF ? NQ : 1];  // MF: the B operand H[e][21 ex + q] (Hᵀ rows >= F are zero)
  const double* hbl = reinterpret_cast<const double*>(smem + wa::L_HT) + NQ * ex * KK + e;  // MFL: from LDS
  // MX: lane (sm, gm); the phase-1 A operand H[l % 4][4ks + gm] (registers at one workgroup per CU,
  // else LDS per tile), the FCLS A operands (table rows) and the validity of the lane's four masks
  const int sm = l & 15, gm = l >> 4;
  constexpr bool MXR = MX && OCC == 1;
  double hx[MXR ? NQ : 1];
  const double* hxl = reinterpret_cast<const double*>(smem + wa::L_HT) + 4 * gm + (l & 3);  // + 16·ks
  // the FCLS A operands (table rows) and the validity of the lane's four masks, per iteration
  double tx[MX ? 4 : 1];
  bool vx[MX ? 4 : 1];
  auto load_h = [&]() {
    if constexpr (MX) {
      if constexpr (MXR) {
#pragma unroll
        for (int ks = 0; ks < NQ; ++ks) hx[ks] = hxl[16 * ks];
      }
#pragma unroll
      for (int bp = 0; bp < 4; ++bp) {
        const int i = l & 15;
        tx[bp] = sTab[(4 * bp + (i & 3)) * wa::TSTR + (((i >> 2) ^ (i & 3)) << 2) + gm];
        vx[bp] = sTab[16 * wa::TSTR + 4 * bp + gm] != 0.0;
      }
    }
    if constexpr (HREG) {
#pragma unroll
      for (int c = 0; c < NQ; ++c)
#pragma unroll
        for (int j = 0; j < KK; ++j) hreg[c][j] = sHtl[c * KK + j];
    }
    if constexpr (MF && !MFL) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) hb[q] = hbl[q * KK];
    }
  };
  load_h();

  f2 acc[NQ][KP], accB[KP];
  auto zero_acc = [&]() {
#pragma unroll
    for (int c = 0; c < NQ; ++c)
#pragma unroll
      for (int p = 0; p < KP; ++p) acc[c][p] = f2{0.f, 0.f};
#pragma unroll
    for (int p = 0; p < KP; ++p) accB[p] = f2{0.f, 0.f};
  };
  zero_acc();

  auto prefetch = [&](u32x4 (&pf)[PFS], int64_t tile) {
    const unsigned char* xs = Xb + (size_t)tile * XBW + 16 * l;
#pragma unroll
    for (int u = 0; u < PFW - 1; ++u) ld16(pf[u], xs + 1024 * u);
    ld16(pf[PFW - 1], l < LASTL ? xs + 1024 * (PFW - 1) : xs);
    if constexpr (TOL || WARM) ld16(pf[PFW], l < 16 ? Wb + (size_t)tile * 256 + 16 * l : xs);  // the tile's W
  };
  auto stage = [&](const u32x4 (&pf)[PFS]) {
    const unsigned addr = (unsigned)(uintptr_t)(stg + 16 * l);
    stage_rec<0, PFW - 1>(addr, pf);
    if (l < LASTL) st16<1024 * (PFW - 1)>(addr, pf[PFW - 1]);
    if constexpr (TOL || WARM)
      if (l < 16) st16<0>((unsigned)(uintptr_t)(wstg + 16 * l), pf[PFW]);
  };

  u32x4 pf[PD][PFS];
  // every body stores its W tile (one store): after each of the first PD sets one dummy store (to this
  // workgroup's partial row, rewritten at the iteration's end) keeps the count of younger operations
  // at a step's wait exact from the first set on (mu_iter_wt_kernel's streamed-W rule).  TOL: the W
  // tile a set loads was stored >= PD steps before (the host keeps nbt >= 2·PD + 1), and the loss
  // iterations' snapshot stores only add younger operations (the waits get stricter, never short).
  float* dummy = reinterpret_cast<float*>(a.partials + (size_t)b * NOUTT) + 64 * w + l;
#pragma unroll
  for (int k = 0; k < PD; ++k) {
    prefetch(pf[k], gw + (int64_t)NW * k);  // the host keeps nbt > PD
    asm volatile("global_store_dword %0, %1, off" ::"v"(dummy), "v"(0) : "memory");
  }
  TL_START;

  bool alive = true;
  // steps per iteration: the wave's nbt tiles padded to a multiple of PD, so that every iteration
  // starts on register set 0 and the end-of-iteration code (reduction, H-step) is emitted ONCE,
  // inlined under the kernel's register budget, after the unrolled streaming loop.  A pad step
  // re-loads the wave's first tile into its set and stores one dummy word (the step's wait counts
  // one store per step).
  const int nbp = (nbt + PD - 1) / PD * PD;
  int nx_i = PD;  // step (within its iteration) whose tile the next prefetch loads
  auto step = [&](u32x4 (&pfk)[PFS]) {
    // younger than this set's loads: the PD - 1 later sets and the stores of the PD steps since
    wait_set<PFS * (PD - 1) + PD, PFS>(pfk);
    stage(pfk);
    prefetch(pfk, gw + (int64_t)NW * (nx_i < nbt ? nx_i : 0));
    if (++nx_i == nbp) nx_i = 0;
  };
  // the wave's exchange scratch (best objective / mask, the new W row): its reduction rows, free
  // while the tiles stream (the x slot stays intact for phase 3); phase 3's lane roles
  unsigned char* xscr = reinterpret_cast<unsigned char*>(red + w * NL * NACC);
  const int s4 = l & 3, g3 = l >> 2;
  const int f5 = g3 + 80 < wa::F ? g3 + 80 : wa::F - 1;  // the 6th feature (g3 = 0 only; else masked)
  const float v5 = g3 + 80 < wa::F ? 1.f : 0.f;
  auto wbody_mx = [&](int i) {
    const int64_t tile = gw + (int64_t)NW * i;
    const float* xr = reinterpret_cast<const float*>(stg) + sm * wa::F + gm;
    // phase 1: c[g][s] on lane (s, g); three accumulation chains summed in a fixed order
    float xv[NQ];
#pragma unroll
    for (int ks = 0; ks < NQ; ++ks) xv[ks] = xr[4 * ks];
    double m0 = 0.0, m1 = 0.0, m2 = 0.0;
    auto hq = [&](int ks) { return MXR ? hx[MXR ? ks : 0] : hxl[16 * ks]; };
#pragma unroll
    for (int ks = 0; ks < NQ; ks += 3) {
      m0 = __builtin_amdgcn_mfma_f64_4x4x4f64(hq(ks), (double)xv[ks], m0, 0, 0, 0);
      if (ks + 1 < NQ) m1 = __builtin_amdgcn_mfma_f64_4x4x4f64(hq(ks + 1), (double)xv[ks + 1], m1, 0, 0, 0);
      if (ks + 2 < NQ) m2 = __builtin_amdgcn_mfma_f64_4x4x4f64(hq(ks + 2), (double)xv[ks + 2], m2, 0, 0, 0);
    }
    const double cs = ((m0 + m1) + m2) + a.delta2;  // c[gm][sm] + δ²
    // c rotated: cr[ρ] = c[gm ^ ρ][sm], the lanes l ^ 16ρ (permlane swaps; round 4 used an identity
    // block on the matrix cores: one 64-cycle f64 MFMA and eight AGPR reads per tile)
    f64x4 cr;
    cr[0] = cs;
    cr[1] = lane_xor16(cs);
    cr[2] = lane_xor32(cs);
    cr[3] = lane_xor32(cr[1]);
    if constexpr (TOL) {
      if ((it0 + cur_it) % 10 == 0) {
        // a loss iteration: ‖x − w·H‖² of the state after it0 + cur_it iterations, per sample as
        // ‖x‖² − 2 w·(Hx) + wᵀ(HHᵀ)w in fp64 (W_g: the tile's W as loaded with X; Hx = c − δ² of
        // the pass, H_g's Gram in LDS — the terms agree to ~1e-11 of the residual at a 1e-5 fit,
        // below the test's 1e-4 steps): ‖x‖² over the lane's features, the rest on lane g = 0,
        // whose rotation is the identity.  W_g's copy goes to the snapshot buffer (a stop here
        // hands the host W_g).
        const float4 wo = *reinterpret_cast<const float4*>(wstg + 16 * sm);
        int so = 4 * sm + gm;  // (opaque: recomputed here, not a loop-invariant 64-bit address)
        asm volatile("" : "+v"(so));
        wsnap[(size_t)tile * (16 * KK) + so] = gm == 0 ? wo.x : (gm == 1 ? wo.y : (gm == 2 ? wo.z : wo.w));
        double xx = 0.0;
#pragma unroll
        for (int ks = 0; ks < NQ; ++ks) {
          const double xd = 4 * ks + gm < wa::F ? (double)xv[ks] : 0.0;
          xx = fma(xd, xd, xx);
        }
        if (gm == 0) {
          const double* hh = reinterpret_cast<const double*>(smem + wa::L_HHT);
          const double w4[4] = {(double)wo.x, (double)wo.y, (double)wo.z, (double)wo.w};
          double cross = 0.0, quad = 0.0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            cross = fma(w4[q], cr[q] - a.delta2, cross);
            double hw = 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) hw = fma(hh[4 * q + r], w4[r], hw);
            quad = fma(w4[q], hw, quad);
          }
          xx = fma(-2.0, cross, xx + quad);
        }
        *lacc += xx;
      }
    }
    // WARM (round 5): the sample's previous passive set P = {j : w_j > 0} (its W as loaded with X)
    // solved first, w_P = (Q_PP)⁻¹ c_P from the table, and certified by the KKT conditions of the
    // strictly convex problem — w_P >= 0 and the dual (Q w − c)_j >= 0 off P — which make it THE
    // minimiser the enumeration below finds (same formula, same bits when it picks the same mask).
    // Only a tile with a sample whose set changed (or whose mask is invalid) runs the enumeration.
    float* xw_ = reinterpret_cast<float*>(xscr + 768);  // the sample rows of the new W (phase 3)
    double wn64;
    bool warm_ok = false;
    if constexpr (WARM) {
      const float4 wo = *reinterpret_cast<const float4*>(wstg + 16 * sm);
      const int mw = (wo.x > 0.f ? 1 : 0) | (wo.y > 0.f ? 2 : 0) | (wo.z > 0.f ? 4 : 0) | (wo.w > 0.f ? 8 : 0);
      const double* T = sTab + mw * wa::TSTR + 4 * gm;
      const double wg = fma(T[gm ^ 3], cr[3], fma(T[gm ^ 2], cr[2], fma(T[gm ^ 1], cr[1], T[gm] * cr[0])));
      const double* Q = reinterpret_cast<const double*>(smem + wa::L_HHT) + 4 * gm;  // HHᵀ row gm
      const double w1 = lane_xor16(wg), w2 = lane_xor32(wg), w3 = lane_xor32(w1);  // w[gm ^ ρ]
      const double dual = fma(Q[gm ^ 3] + a.delta2, w3, fma(Q[gm ^ 2] + a.delta2, w2,
                              fma(Q[gm ^ 1] + a.delta2, w1, (Q[gm] + a.delta2) * wg))) - cs;
      const bool inP = ((mw >> gm) & 1) != 0;
      const bool ok = sTab[16 * wa::TSTR + mw] != 0.0 && (inP ? wg >= 0.0 : dual >= 0.0);
      warm_ok = __ballot(!ok) == 0;  // wave-uniform
      wn64 = wg;
    }
    if (!warm_ok) {
    // FCLS: the 16 masks' solutions, lane (s, g) block b' = mask 4b' + g (register ρ = component ρ ^ g);
    // the lane's masks ascend with b', so a strict < keeps the lowest of tied masks
    double bestf = 1.0;
    int bestm = 16;
#pragma unroll
    for (int bp = 0; bp < 4; ++bp) {
      const f64x4 v = __builtin_amdgcn_mfma_f64_16x16x4f64(tx[bp], cs, f64x4{0.0, 0.0, 0.0, 0.0}, 0, 0, 0);
      const bool feas = vx[bp] & (v[0] >= 0.0) & (v[1] >= 0.0) & (v[2] >= 0.0) & (v[3] >= 0.0);
      const double f = -0.5 * fma(cr[3], v[3], fma(cr[2], v[2], fma(cr[1], v[1], cr[0] * v[0])));
      const bool take = feas & (f < bestf);
      bestf = take ? f : bestf;
      bestm = take ? 4 * bp + gm : bestm;
    }
    // the sample's four lanes exchange their best through the wave's staging slot (its x is in
    // registers; in-order LDS inside the wave) and each takes the least (objective, mask)
    double* xf_ = reinterpret_cast<double*>(xscr);
    int* xm_ = reinterpret_cast<int*>(xscr + 512);
    xf_[4 * sm + gm] = bestf;
    xm_[4 * sm + gm] = bestm;
    {
      const double4 fo = *reinterpret_cast<const double4*>(xf_ + 4 * sm);
      const int4 mo = *reinterpret_cast<const int4*>(xm_ + 4 * sm);
      auto pick = [&](double f2_, int m2_) {
        const bool tk = (f2_ < bestf) | ((f2_ == bestf) & (m2_ < bestm));
        bestf = tk ? f2_ : bestf;
        bestm = tk ? m2_ : bestm;
      };
      bestf = fo.x;
      bestm = mo.x;
      pick(fo.y, mo.y);
      pick(fo.z, mo.z);
      pick(fo.w, mo.w);
    }
    {
      const double* T = sTab + min(bestm, 15) * wa::TSTR + 4 * gm;
      wn64 = fma(T[gm ^ 3], cr[3], fma(T[gm ^ 2], cr[2], fma(T[gm ^ 1], cr[1], T[gm] * cr[0])));
    }
    }  // the enumeration
    const float wn = (float)fmax(wn64, 0.0);
    // the tile's 256 contiguous bytes (the lane's offset opaque: TOL kept the 64-bit lane address
    // across the iteration loop, spilled, and reloaded it behind a vmcnt(0) at every iteration)
    a.W[(size_t)tile * (16 * KK) + opaque_i(4 * sm + gm)] = wn;
    // phase 3, regrouped: lane (s4 = l % 4, g3 = l / 4) takes the tile's samples 4j + s4 (j < 4) and
    // the features g3 + 16k (k < 6; k = 5 only for g3 = 0), x read again from the slot: 24 + 4 fp32
    // accumulators per lane instead of the (s, g) layout's 88 and no x registers across the FCLS —
    // the streaming loop then keeps every value in registers (a spill reload there waits on, and
    // drains, the prefetch)
    xw_[4 * sm + gm] = wn;
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      const int s3 = 4 * j4 + s4;
      const float4 w4 = *reinterpret_cast<const float4*>(xw_ + 4 * s3);
      const float wr = xw_[4 * s3 + (g3 & 3)];
      const f2 wp0 = f2{w4.x, w4.y}, wp1 = f2{w4.z, w4.w};
      const float* xs3 = reinterpret_cast<const float*>(stg) + wa::F * s3;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        float xx1 = xs3[k < 5 ? g3 + 16 * k : f5];
        if (k == 5) xx1 *= v5;
        const f2 xx = f2{xx1, xx1};
        acc[k][0] = __builtin_elementwise_fma(xx, wp0, acc[k][0]);
        acc[k][1] = __builtin_elementwise_fma(xx, wp1, acc[k][1]);
      }
      accB[0] = __builtin_elementwise_fma(f2{wr, wr}, wp0, accB[0]);
      accB[1] = __builtin_elementwise_fma(f2{wr, wr}, wp1, accB[1]);
    }
  };
  auto wbody = [&](int i) {
    if constexpr (MX) {
      wbody_mx(i);
      return;
    }
    const int64_t tile = gw + (int64_t)NW * i;
    // phase 1: c = H·x over the lane's features in fp64, quad butterfly, + δ²
    const float* xr = reinterpret_cast<const float*>(stg) + sx * wa::F + NQ * ex;
    float xv[NQ];
#pragma unroll
    for (int c = 0; c < NQ; ++c) xv[c] = xr[c];
    double cc[KK] = {0.0, 0.0, 0.0, 0.0};
    if constexpr (MF) {
      // three accumulation chains (the MFMA's dependent latency), summed in a fixed order
      double m0 = 0.0, m1 = 0.0, m2 = 0.0;
      auto hbq = [&](int q) { return MFL ? hbl[q * KK] : hb[MFL ? 0 : q]; };
#pragma unroll
      for (int q = 0; q < NQ; q += 3) {
        m0 = __builtin_amdgcn_mfma_f64_4x4x4f64((double)xv[q], hbq(q), m0, 0, 0, 0);
        if (q + 1 < NQ) m1 = __builtin_amdgcn_mfma_f64_4x4x4f64((double)xv[q + 1], hbq(q + 1), m1, 0, 0, 0);
        if (q + 2 < NQ) m2 = __builtin_amdgcn_mfma_f64_4x4x4f64((double)xv[q + 2], hbq(q + 2), m2, 0, 0, 0);
      }
      const double cs = ((m0 + m1) + m2) + a.delta2;  // c[s][e] + δ² on lane 4s + e
      cc[0] = dpp64<0x00>(cs);                         // quad broadcasts: lane 4s + j's value
      cc[1] = dpp64<0x55>(cs);
      cc[2] = dpp64<0xAA>(cs);
      cc[3] = dpp64<0xFF>(cs);
    } else {
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      const double2 h01 = HREG ? make_double2(hreg[HREG ? c : 0][0], hreg[HREG ? c : 0][1])
                               : *reinterpret_cast<const double2*>(sHtl + c * KK);
      const double2 h23 = HREG ? make_double2(hreg[HREG ? c : 0][2], hreg[HREG ? c : 0][3])
                               : *reinterpret_cast<const double2*>(sHtl + c * KK + 2);
      const double x = (double)xv[c];
      cc[0] = fma(x, h01.x, cc[0]);
      cc[1] = fma(x, h01.y, cc[1]);
      cc[2] = fma(x, h23.x, cc[2]);
      cc[3] = fma(x, h23.y, cc[3]);
    }
#pragma unroll
    for (int j = 0; j < KK; ++j) cc[j] += dpp64<0xB1>(cc[j]);  // quad_perm [1,0,3,2]: + lane ^ 1
#pragma unroll
    for (int j = 0; j < KK; ++j) cc[j] = cc[j] + dpp64<0x4E>(cc[j]) + a.delta2;  // [2,3,0,1]: + lane ^ 2
    }
    // FCLS: the passive sets e, e + 4, e + 8, e + 12
    double bestf = 1.0;
    int bestm = 16;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = e + 4 * u;
      const double* T = sTab + m * wa::TSTR;
      bool feas = sTab[16 * wa::TSTR + m] != 0.0;
      double f = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) v = fma(T[r * 4 + q], cc[q], v);
        feas = feas && v >= 0.0;
        f = fma(cc[r], v, f);
      }
      f *= -0.5;
      if (feas && (f < bestf || (f == bestf && m < bestm))) {
        bestf = f;
        bestm = m;
      }
    }
#pragma unroll
    for (int off = 1; off <= 2; off <<= 1) {
      const double of = __shfl_xor(bestf, off);
      const int om = __shfl_xor(bestm, off);
      if (of < bestf || (of == bestf && om < bestm)) {
        bestf = of;
        bestm = om;
      }
    }
    double wn64 = 0.0;
    {
      const double* T = sTab + min(bestm, 15) * wa::TSTR;
#pragma unroll
      for (int q = 0; q < 4; ++q) wn64 = fma(T[e * 4 + q], cc[q], wn64);
    }
    const float wn = (float)fmax(wn64, 0.0);
    a.W[(size_t)tile * (16 * KK) + l] = wn;  // lane l = (s, e): the tile's 256 contiguous bytes
    // phase 3 with the sample's new row: quad broadcasts, or (MF) the row of sample sx through the
    // wave's staging slot (its X was read above: in-order LDS inside the wave)
    f2 wp[KP];
    float wk = wn;  // B[ex][·] += w'[ex]·w'
    if constexpr (MF) {
      reinterpret_cast<float*>(stg)[l] = wn;
      const float4 wq = *reinterpret_cast<const float4*>(stg + 16 * sx);
      wp[0] = f2{wq.x, wq.y};
      wp[1] = f2{wq.z, wq.w};
      wk = ex == 0 ? wq.x : (ex == 1 ? wq.y : (ex == 2 ? wq.z : wq.w));
    } else {
      wp[0] = f2{dppf<0x00>(wn), dppf<0x55>(wn)};
      wp[1] = f2{dppf<0xAA>(wn), dppf<0xFF>(wn)};
    }
#pragma unroll
    for (int c = 0; c < NQ; ++c) {
      const f2 xx = f2{xv[c], xv[c]};
#pragma unroll
      for (int q = 0; q < KP; ++q) acc[c][q] = __builtin_elementwise_fma(xx, wp[q], acc[c][q]);
    }
#pragma unroll
    for (int q = 0; q < KP; ++q) accB[q] = __builtin_elementwise_fma(f2{wk, wk}, wp[q], accB[q]);
  };
  auto end_iteration = [&](int it) {
    const bool last_it = it + 1 == a.n_iter;
    // the thread's roles recomputed here from an opaque copy of its id (opaque_i)
    const int t = opaque_i(threadIdx.x);
    const int l = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int s4 = l & 3, g3 = l >> 2;
    // ---- end of this wave's iteration: mu_iter_wt_kernel's reduction (k = 4)
    if constexpr (MX) {
      // the quad's four sample groups summed (lanes 4·g3 .. 4·g3 + 3); its first lane writes the
      // features g3 + 16k and, g3 < 4, the WᵀW row g3
      auto qsum = [&](float v) {
        v += dppf<0xB1>(v);         // quad_perm [1,0,3,2]
        return v + dppf<0x4E>(v);   // quad_perm [2,3,0,1]
      };
      const bool wr = s4 == 0;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const float4 v = make_float4(qsum(acc[k][0].x), qsum(acc[k][0].y), qsum(acc[k][1].x), qsum(acc[k][1].y));
        const int f = g3 + 16 * k;
        if (wr && f < wa::F) {
          const int ee = f / NQ;
          *reinterpret_cast<float4*>(red + (w * NL + ee) * NACC + (f - NQ * ee) * KK) = v;
        }
      }
      const float4 v = make_float4(qsum(accB[0].x), qsum(accB[0].y), qsum(accB[1].x), qsum(accB[1].y));
      if (wr && g3 < 4) *reinterpret_cast<float4*>(red + (w * NL + g3) * NACC + NQ * KK) = v;
    } else {
      // the sums over the lanes of one feature group: lanes ≡ e (mod 4), or (MF) the 16 lanes of a row
      auto ssum = [&](float v) { return MF ? sum_over_row16(v) : sum_over_samples<NL>(v); };
      const bool wr = MF ? (l & 15) == 0 : l < NL;
      float* rw = red + (w * NL + ex) * NACC;
#pragma unroll
      for (int c = 0; c < NQ; ++c) {
        const float4 v = make_float4(ssum(acc[c][0].x), ssum(acc[c][0].y), ssum(acc[c][1].x), ssum(acc[c][1].y));
        if (wr) *reinterpret_cast<float4*>(rw + c * KK) = v;
      }
      const float4 v = make_float4(ssum(accB[0].x), ssum(accB[0].y), ssum(accB[1].x), ssum(accB[1].y));
      if (wr) *reinterpret_cast<float4*>(rw + NQ * KK) = v;
    }
    zero_acc();
    const bool loss_it = TOL && ((it0 + it) % 10 == 0);  // this iteration checked the state after it0 + it
    if constexpr (TOL) {  // the wave's loss sum (zero outside loss iterations), fixed xor tree
      const double v = wave_sum(*lacc);
      if (l == 0) sLoss[w] = v;
      *lacc = 0.0;
    }
    __syncthreads();
    {
      double* prow = a.partials + (size_t)b * NOUTT;
      if (TOL && t == 0)
        __hip_atomic_store(prow + NOUT, (sLoss[0] + sLoss[1]) + (sLoss[2] + sLoss[3]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      auto row_val = [&](int o) {
        const int j = o / V;
        const int v = o - j * V;
        const int ee = v < wa::F ? v / NQ : j;
        const int idx = v < wa::F ? (v - NQ * ee) * KK + j : NQ * KK + (v - wa::F);
        const float* rr = red + ee * NACC + idx;
        constexpr int WS = NL * NACC;
        return ((double)rr[0] + (double)rr[WS]) + ((double)rr[2 * WS] + (double)rr[3 * WS]);
      };
      if constexpr (VT) {  // pairs of doubles, one 16-byte sc1 store each (round 6)
        if (t < NOUT / 2) st16_sc1v(prow + 2 * t, row_val(2 * t), row_val(2 * t + 1));
      } else {
        for (int o = t; o < NOUT; o += NT) __hip_atomic_store(prow + o, row_val(o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    TL(it, 0);
    if (t == 0) {
      const uint32_t old = __hip_atomic_fetch_add(cnt_group, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sFlag[0] = old == (uint32_t)((it + 1) * gs - 1);
      sFlag[1] = 0;
      sFlag[2] = 1;
      sFlag[3] = 0;
    }
    __syncthreads();
    // TOL: the last iteration of the launch waits for the flag too when it checks the tolerance (a
    // stop there must reach every workgroup before the top applies the last H-step)
    const bool must_wait = !last_it || loss_it;
    if (sFlag[0]) {  // group combiner
      if constexpr (VT) sum_rows_v<NOUTT>(a.partials, g, NG, gs, nullptr, a.groups + (size_t)g * NOUTT, t);
      else sum_rows_n<NOUTT>(a.partials, g, NG, gs, nullptr, a.groups + (size_t)g * NOUTT, t);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) {
        const uint32_t old = __hip_atomic_fetch_add(cnt_top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sFlag[1] = old == (uint32_t)((it + 1) * NG - 1);
      }
      __syncthreads();
      if (sFlag[1]) {  // top combiner: AB
        if constexpr (VT) {
          sum_rows_v<NOUTT>(a.groups, 0, 1, NG, sAB, a.AB, t);
          if (MULTI) __syncthreads();  // the exchange reads sAB in sum_rows_n's thread mapping
        } else {
          sum_rows_n<NOUTT>(a.groups, 0, 1, NG, sAB, a.AB, t);
        }
        if (MULTI) xchg_allreduce_n<NOUTT>(a.xctl, a.AB, sAB, err, it, t);  // + the other ranks' AB
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (TOL && loss_it && t == 0) {  // the relative-decrease test on the state after it0 + it
          const int gi = it0 + it;
          const double errv = sqrt(fmax(sAB[NOUT], 0.0));
          const int slot = gi / 10;
          if (slot < (int)ld_sc1(a.tolctl + TC_CAP)) st_sc1(a.tolctl + TC_ERRS + slot, errv);
          st_sc1(a.tolctl + TC_NERR, (double)(slot + 1));
          if (gi == 0) {
            sLoss[4] = sLoss[5] = errv;
            st_sc1(a.tolctl + TC_INIT, errv);
            st_sc1(a.tolctl + TC_PREV, errv);
          } else if ((sLoss[5] - errv) / sLoss[4] < sLoss[6]) {
            sFlag[3] = 1;
          } else {
            sLoss[5] = errv;
            st_sc1(a.tolctl + TC_PREV, errv);
          }
        }
        if (TOL && loss_it) __syncthreads();  // sFlag[3] (the decision) for the whole workgroup
        if (t == 0 && must_wait)
          __hip_atomic_store(flag, (uint32_t)(it + 1) | (sFlag[3] ? FLAG_STOP : 0u), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        TL_PUB(it);
      }
    }
    const bool top = sFlag[1] != 0;
    if (!top && must_wait) {
      if (t == 0) {
        const uint32_t want = (uint32_t)(it + 1);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t f;
        while (true) {  // the flag and the error word in one batch: one round trip per round
          const uint32_t ev = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((f & ~FLAG_STOP) >= want) break;
          if (ev != 0u) {
            sFlag[2] = 0;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > sl::SPIN_TIMEOUT) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sFlag[2] = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (TOL && (f & FLAG_STOP)) sFlag[3] = 1;
      }
      __syncthreads();
      if (!sFlag[2]) {
        alive = false;
        return;
      }
    }
    if (!last_it) PH(0);
    // the basis state for the host (the last combiner of the launch, or the top of a stop)
    auto write_state = [&]() {
      for (int o = t; o < KK * wa::F; o += NT) a.H64[o] = sH[o];
      for (int o = t; o < wa::F * KK; o += NT) a.Ht[o] = reinterpret_cast<const double*>(smem + wa::L_HT)[o];
      if (t < KK * KK) a.HHt[t] = reinterpret_cast<const double*>(smem + wa::L_HHT)[t];
      for (int o = t; o < ALS_TAB; o += NT)  // the global table keeps the stride of 16
        a.table[o] = o < 256 ? sTab[(o >> 4) * wa::TSTR + (o & 15)] : sTab[16 * wa::TSTR + (o - 256)];
      if (t < NG) __hip_atomic_store(a.cnt + CNT_GROUP0 + 32 * t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    if (TOL && sFlag[3]) {
      // stopped by the tolerance test: the state after it0 + it iterations — H_g (this iteration's
      // H-step not applied), W_g in the snapshot buffer; the host clears the flag word
      alive = false;
      if (!top) return;
      write_state();
      if (t == 0) {
        __hip_atomic_store(cnt_top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st_sc1(a.tolctl + TC_DONE, (double)(it0 + it));
        st_sc1(a.tolctl + TC_STOPPED, 1.0);
        st_sc1(a.tolctl + TC_IN_SNAP, 1.0);
        if (MULTI)
          __hip_atomic_fetch_add(a.xctl + XC_GEN, (uint64_t)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (last_it) {
      alive = false;
      if (!top) return;
      // the last combiner of the launch: the last H-step, then the basis state for the host
      wa_update_basis(t, opaque_d(a.lam), opaque_d(a.delta2), true);
      write_state();
      if (t == 0) {
        __hip_atomic_store(cnt_top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!must_wait)  // (else workgroups may still poll it: the host clears it after the launch)
          __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (TOL) {
          st_sc1(a.tolctl + TC_DONE, (double)(it0 + a.n_iter));
          st_sc1(a.tolctl + TC_STOPPED, 0.0);
        }
        if (MULTI)  // the next launch's generations follow this one's
          __hip_atomic_fetch_add(a.xctl + XC_GEN, (uint64_t)a.n_iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (!top) {
      // AB straight into the H-step's A / B arrays (TOL's loss slot into sAB)
      double* hA = reinterpret_cast<double*>(smem + wa::L_HS);
      auto put = [&](int o, double v) {
        const int j = o / V, c = o - j * V;
        if (o >= NOUT) sAB[o] = v;
        else if (c < wa::F) hA[j * wa::F + c] = v;
        else hA[2 * KK * wa::F + j * KK + (c - wa::F)] = v;
      };
      if constexpr (VT) {  // one 16-byte sc1 load per thread (round 6)
        u32x4 r;
        ld16_sc1(r, a.AB + 2 * (t < NOUT / 2 ? t : 0));
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(r) : : "memory");
        if (t < NOUT / 2) {
          put(2 * t, lo_d(r));
          put(2 * t + 1, hi_d(r));
        }
      } else {
        for (int o = t; o < NOUTT; o += NT) put(o, ld_sc1(a.AB + o));
      }
      __syncthreads();
      if (TOL && loss_it && t == 0) {  // the top went on: prev <- this check's error
        const double errv = sqrt(fmax(sAB[NOUT], 0.0));
        if (it0 + it == 0) sLoss[4] = errv;
        sLoss[5] = errv;
      }
    }
    PH(1);
    wa_update_basis(t, opaque_d(a.lam), opaque_d(a.delta2), top);
    load_h();
    PH(7);
    TL(it, 1);
  };

  for (int it = 0; it < a.n_iter && alive; ++it) {
    cur_it = it;
    for (int i0 = 0; i0 < nbp; i0 += PD) {
      if (a.prio) {
        // the ladder: a wave with more steps left issues first, so the two workgroups sharing a CU
        // (each SIMD runs one wave of each) finish their iteration together instead of the older one
        // first and the younger alone at one wave per SIMD
        const int rem = nbp - i0;
        if (rem > 3 * a.prio) __builtin_amdgcn_s_setprio(3);
        else if (rem > 2 * a.prio) __builtin_amdgcn_s_setprio(2);
        else if (rem > a.prio) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
#pragma unroll
      for (int k = 0; k < PD; ++k) {
        step(pf[k]);
        if (i0 + k < nbt) wbody(i0 + k);
        else asm volatile("global_store_dword %0, %1, off" ::"v"(dummy), "v"(0) : "memory");
      }
    }
    end_iteration(it);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the workgroup
}

// tile size of the weighted pass: the largest of 64 / 32 / 16 / 8 samples whose LDS fits 64 KB
static int wmu_tile(int F, int KP) {
  for (int ts = 64; ts >= 8; ts >>= 1) {
    const size_t lds = ((size_t)(2 * ts * F + KP * F + 2 * ts * KP) * 4 + 15) / 16 * 16 + NWAVE * 8;
    if (lds <= 64 * 1024 && ts * F <= 4 * NT * WMU_MAXC) return ts;
  }
  return 0;
}
static size_t wmu_lds(int F, int KP, int ts) {
  return ((size_t)(2 * ts * F + KP * F + 2 * ts * KP) * 4 + 15) / 16 * 16 + NWAVE * 8;
}
// partial rows per workgroup: 1 when the phase-2 groups' sums fold in the pass's own LDS, else one
// per group (the reduction then sums them)
static int wmu_rows(int F, int k) {
  const int g2 = F <= NT ? NT / F : 1;
  if (g2 == 1) return 1;
  const int KP = k <= 4 ? 4 : 8;
  const int ts = wmu_tile(F, KP);
  return (size_t)g2 * 2 * k * F * 8 <= wmu_lds(F, KP, ts) ? 1 : g2;
}
static constexpr int64_t kWmuMaxBlocks = 512;  // two per CU resident (occupancy 2 waves / SIMD)

extern "C" {

int cnmf_abi_version(void) { return 302; }

const char* cnmf_last_error(void) { return g_err; }

int cnmf_padded_k(int k) { return (k < 1 || k > 16) ? -1 : padded_k(k); }

int64_t cnmf_stage_doubles(int n_out) { return (int64_t)NSLICE * (n_out > 0 ? n_out : 1); }

// Grid of the accumulating pass.  For the sample-lane pass: its workgroups over the full tiles plus
// one workgroup of mu_pass_kernel for a ragged tail (its partial row is the last one).
static int64_t sl_grid(int64_t n_rows, int64_t* n_full, bool* tail) {
  *n_full = n_rows / TS;
  *tail = (n_rows % TS) != 0;
  int64_t g = 0;
  if (*n_full > 0) {
    g = pass_grid(*n_full * TS, reinterpret_cast<PassFn>(&mu_pass_sl_kernel), sl::L_TOTAL);
    if (g < 0) return -1;
  }
  return g;
}

static int64_t main_grid(int64_t n_rows, int x_dtype, int F, int k, PassKernel* pk, size_t* lds) {
  if (use_bfw(x_dtype, F, k)) {  // the wave-tile grid over the full tiles, + one row for a ragged tail
    const int64_t n_full = n_rows / TS;
    int64_t g = 0;
    if (n_full > 0) {
      g = pass_grid(n_full * TS, bfw_fn(F, k), (size_t)bw::lds(F).total);
      if (g < 0) return -1;
    }
    return g + (n_rows % TS != 0 ? 1 : 0);
  }
  if (use_sl(x_dtype, F, k)) {
    int64_t n_full;
    bool tail;
    const int64_t g = sl_grid(n_rows, &n_full, &tail);
    return g < 0 ? -1 : g + (tail ? 1 : 0);
  }
  return pass_grid(n_rows, pk->fn, *lds);
}

int64_t cnmf_pass_blocks(int64_t n_rows, int n_features, int k, int x_dtype) {
  if (n_rows < 0) return set_err(CNMF_ERR_SHAPE, "n_rows < 0");
  PassKernel pk;
  size_t lds = 0;
  int st = select_pass(x_dtype, n_features, k, &pk, &lds);
  if (st) return st;
  int64_t nb = main_grid(n_rows, x_dtype, n_features, k, &pk, &lds);
  if (nb < 0) return set_err(CNMF_ERR_HIP, "occupancy query failed (no HIP device?)");
  return nb;
}

int cnmf_mu_sample_pass(const void* X, int x_dtype, void* W, const double* Ht, const double* HHt,
                        double* partials, int64_t n_rows, int n_features, int k, double l1_W,
                        double l2_W, int flags, void* stream) {
  if (n_rows < 0) return set_err(CNMF_ERR_SHAPE, "n_rows < 0");
  if (!X || !W || !Ht || !HHt) return set_err(CNMF_ERR_ARG, "null pointer argument");
  const int valid = CNMF_PASS_UPDATE_W | CNMF_PASS_ACCUMULATE | CNMF_PASS_LOSS;
  if ((flags & ~valid) || flags == 0 || ((flags & CNMF_PASS_LOSS) && flags != CNMF_PASS_LOSS) ||
      ((flags & CNMF_PASS_ACCUMULATE) && !(flags & CNMF_PASS_UPDATE_W)))
    return set_err(CNMF_ERR_ARG, "invalid flags %d", flags);
  if ((flags & (CNMF_PASS_ACCUMULATE | CNMF_PASS_LOSS)) && !partials)
    return set_err(CNMF_ERR_ARG, "partials required");
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(W) & 15))
    return set_err(CNMF_ERR_ALIGN, "X and W must be 16-byte aligned");
  // every launch of a shape uses the grid of its main (accumulating) kernel, so the number of
  // partial rows is one per shape (cnmf_pass_blocks) whatever the flags
  PassKernel pmain;
  size_t lmain = 0;
  int st = select_pass(x_dtype, n_features, k, &pmain, &lmain);
  if (st) return st;
  const int64_t nb = main_grid(n_rows, x_dtype, n_features, k, &pmain, &lmain);
  if (nb < 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
  if (nb == 0) return CNMF_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int F = n_features;
  const bool sl_path = use_sl(x_dtype, n_features, k);
  if (sl_path && flags == (CNMF_PASS_UPDATE_W | CNMF_PASS_ACCUMULATE)) {
    int64_t n_full;
    bool tail;
    const int64_t g = sl_grid(n_rows, &n_full, &tail);
    if (g > 0) {
      hipLaunchKernelGGL(mu_pass_sl_kernel, dim3((unsigned)g), dim3(NT), sl::L_TOTAL, s,
                         static_cast<const float*>(X), static_cast<float*>(W), Ht, HHt, partials,
                         n_full, l1_W, l2_W);
      HIP_CHECK(hipGetLastError());
    }
    if (!tail) return CNMF_OK;
    // the ragged tail (< 64 rows) on one workgroup of the VALU pass, partial row g
    PassKernel pk;
    size_t lds = 0;
    st = select_pass(x_dtype, n_features, k, &pk, &lds, false);
    if (st) return st;
    if (max_resident(pk.fn, lds) <= 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
    const void* Xt = static_cast<const float*>(X) + n_full * TS * F;
    void* Wt = static_cast<float*>(W) + n_full * TS * k;
    double* pt = partials + g * (int64_t)k * (F + k);
    int64_t rows = n_rows - n_full * TS, one = 1;
    void* args[] = {(void*)&Xt, &Wt, (void*)&Ht, (void*)&HHt, &pt, &rows, &F, &k, &l1_W, &l2_W, &flags, (void*)&one};
    HIP_CHECK(hipLaunchKernel(pk.fn, dim3(1), dim3(NT), args, lds, s));
    return CNMF_OK;
  }
  if (use_bfw(x_dtype, n_features, k) && (flags & CNMF_PASS_UPDATE_W) && partials) {
    const int64_t n_full = n_rows / TS;
    int64_t g = 0;
    if (n_full > 0) {
      const size_t lb = (size_t)bw::lds(F).total;
      g = pass_grid(n_full * TS, bfw_fn(F, k), lb);
      if (g <= 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
      int64_t nt = n_full;
      void* args[] = {(void*)&X, &W, (void*)&Ht, (void*)&HHt, &partials, &n_rows, &F, &k, &l1_W, &l2_W, &flags, (void*)&nt};
      HIP_CHECK(hipLaunchKernel(bfw_fn(F, k), dim3((unsigned)g), dim3(NT), args, lb, s));
    }
    if (n_rows % TS == 0) return CNMF_OK;
    // the ragged tail (< 64 rows) on one workgroup of the 64-sample matrix-core pass, partial row g
    if (max_resident(pmain.fn, lmain) <= 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
    const void* Xt = static_cast<const bf16_t*>(X) + n_full * TS * F;
    void* Wt = static_cast<float*>(W) + n_full * TS * k;
    double* pt = partials ? partials + g * (int64_t)k * (F + k) : nullptr;
    int64_t rows = n_rows - n_full * TS, one = 1;
    void* args[] = {(void*)&Xt, &Wt, (void*)&Ht, (void*)&HHt, &pt, &rows, &F, &k, &l1_W, &l2_W, &flags, (void*)&one};
    HIP_CHECK(hipLaunchKernel(pmain.fn, dim3(1), dim3(NT), args, lmain, s));
    return CNMF_OK;
  }
  PassKernel pk = pmain;
  size_t lds = lmain;
  if ((flags & CNMF_PASS_LOSS) || sl_path) {
    st = select_pass(x_dtype, n_features, k, &pk, &lds, false);
    if (st) return st;
    if (max_resident(pk.fn, lds) <= 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
  }
  const int64_t n_tiles = (n_rows + TS - 1) / TS;
  void* args[] = {(void*)&X, &W, (void*)&Ht, (void*)&HHt, &partials, &n_rows, &F, &k, &l1_W, &l2_W, &flags, (void*)&n_tiles};
  HIP_CHECK(hipLaunchKernel(pk.fn, dim3((unsigned)nb), dim3(NT), args, lds, s));
  return CNMF_OK;
}

static int launch_reduce(const double* partials, int64_t n_parts, int n_out, double* stage,
                         uint32_t* counter, double* out, int fuse, UpdateArgs ua, hipStream_t s) {
  if (!stage || !counter || !out || (n_parts > 0 && !partials))
    return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (n_out < 1 || n_parts < 0) return set_err(CNMF_ERR_SHAPE, "invalid reduce shape");
  if (!fuse && n_out >= RW_MIN_OUT && n_parts <= RW_MAX_ROWS) {  // wide rows: one level
    // 16 columns per workgroup (8 and 32 measured the same at cfg4, profiles/r06/cfg4_reduce/)
    constexpr int cols = 16;
    hipLaunchKernelGGL(reduce_wide_kernel<cols>, dim3((unsigned)((n_out + cols - 1) / cols)), dim3(RED_NT), 0, s,
                       partials, n_parts, n_out, out);
    HIP_CHECK(hipGetLastError());
    return CNMF_OK;
  }
  const size_t lds = reduce_lds(n_out, fuse, ua.F, ua.k);
  if (lds > kMaxLds) return set_err(CNMF_ERR_UNSUPPORTED, "basis too large for the fused update");
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&reduce_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int nslice = (int)std::max<int64_t>(1, std::min<int64_t>(NSLICE, (n_parts + 4 * RED_ROWS_PER_THREAD - 1) / (4 * RED_ROWS_PER_THREAD)));
  if ((int64_t)nslice * 4 * RED_ROWS_PER_THREAD < n_parts)
    return set_err(CNMF_ERR_UNSUPPORTED, "too many partial rows (%lld) for one reduction", (long long)n_parts);
  if ((n_out + 63) / 64 > RED_MAX_COLS) return set_err(CNMF_ERR_UNSUPPORTED, "n_out=%d too wide for the reduction", n_out);
  dim3 grid((unsigned)((n_out + 63) / 64), (unsigned)nslice);
  hipLaunchKernelGGL(reduce_kernel, grid, dim3(RED_NT), lds, s, partials, n_parts, n_out, nslice,
                     stage, counter, out, fuse, ua);
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}

int cnmf_reduce_partials(const double* partials, int64_t n_parts, int n_out, double* stage,
                         uint32_t* counter, double* out, void* stream) {
  UpdateArgs ua{};
  ua.F = 1;
  ua.k = 1;
  return launch_reduce(partials, n_parts, n_out, stage, counter, out, 0, ua,
                       reinterpret_cast<hipStream_t>(stream));
}

static int check_update_args(const double* H64, const double* Ht, const double* HHt, int F, int k) {
  if (!H64 || !Ht || !HHt) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (F < 1 || k < 1) return set_err(CNMF_ERR_SHAPE, "invalid shape F=%d k=%d", F, k);
  if (k > 16) return set_err(CNMF_ERR_UNSUPPORTED, "k=%d > 16 is not supported", k);
  if (k > 4 && F > 512) return set_err(CNMF_ERR_UNSUPPORTED, "n_features=%d > 512 with k=%d > 4", F, k);
  return CNMF_OK;
}

int cnmf_basis_update(const double* AB, double* H64, double* Ht, double* HHt, int n_features, int k,
                      double l1_H, double l2_H, int do_update, double* stats, void* stream) {
  int st = check_update_args(H64, Ht, HHt, n_features, k);
  if (st) return st;
  if (do_update && !AB) return set_err(CNMF_ERR_ARG, "AB required for do_update");
  const int KP = padded_k(k);
  const size_t lds = update_lds_doubles(n_features, k, KP) * sizeof(double);
  if (lds > kMaxLds) return set_err(CNMF_ERR_UNSUPPORTED, "basis too large for the update kernel");
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&basis_update_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(basis_update_kernel, dim3(1), dim3(RED_NT), lds,
                     reinterpret_cast<hipStream_t>(stream), AB, H64, Ht, HHt, n_features, k, KP, l1_H,
                     l2_H, do_update, stats);
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}

int cnmf_normalise(void* W, int w_dtype, double* H64, double* Ht, double* HHt, double* scale,
                   int64_t n_rows, int n_features, int k, int norm, void* stream) {
  int st = check_update_args(H64, Ht, HHt, n_features, k);
  if (st) return st;
  if (!scale || (n_rows > 0 && !W)) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (norm < 1 || norm > 3) return set_err(CNMF_ERR_ARG, "norm must be 1 (L1), 2 (L2) or 3 (max)");
  if (w_dtype != CNMF_F32 && w_dtype != CNMF_F64) return set_err(CNMF_ERR_ARG, "W must be f32 or f64");
  if (n_rows < 0) return set_err(CNMF_ERR_SHAPE, "n_rows < 0");
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const int KP = padded_k(k);
  const size_t lds = (16 + update_lds_doubles(n_features, k, KP)) * sizeof(double);
  if (lds > kMaxLds) return set_err(CNMF_ERR_UNSUPPORTED, "basis too large for the update kernel");
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&normalise_basis_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(normalise_basis_kernel, dim3(1), dim3(RED_NT), lds, hs, H64, Ht, HHt, scale,
                     n_features, k, KP, norm);
  HIP_CHECK(hipGetLastError());
  const int64_t n = n_rows * k;
  if (n == 0) return CNMF_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>(4096, (n + 255) / 256);
  if (w_dtype == CNMF_F32)
    hipLaunchKernelGGL(scale_columns_kernel<float>, dim3(blocks), dim3(256), 0, hs, static_cast<float*>(W),
                       scale, n, k);
  else
    hipLaunchKernelGGL(scale_columns_kernel<double>, dim3(blocks), dim3(256), 0, hs, static_cast<double*>(W),
                       scale, n, k);
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}

int cnmf_als_table_doubles(void) { return ALS_TAB; }

static int als_basis_launch(const double* AB, double* H64, double* Ht, double* HHt, double* table, int F,
                            int k, double lam, double delta, int do_update, hipStream_t s) {
  int st = check_update_args(H64, Ht, HHt, F, k);
  if (st) return st;
  if (!table || (do_update && !AB)) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (k > ALS_MAX_K) return set_err(CNMF_ERR_UNSUPPORTED, "constrained ALS supports k <= %d (got %d)", ALS_MAX_K, k);
  if (F > ALS_MAX_F) return set_err(CNMF_ERR_UNSUPPORTED, "constrained ALS supports F <= %d", ALS_MAX_F);
  if (!(lam >= 0.0) || !(delta >= 0.0)) return set_err(CNMF_ERR_ARG, "smoothness and sum_to_one must be >= 0");
  const size_t lds = std::max(als_lds_bytes(F, k), update_lds_doubles(F, k, 4) * sizeof(double));
  if (lds > kMaxLds) return set_err(CNMF_ERR_UNSUPPORTED, "basis too large for the ALS update");
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&als_basis_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(als_basis_kernel, dim3(1), dim3(RED_NT), lds, s, AB, H64, Ht, HHt, table, F, k, 4, lam,
                     delta * delta, do_update);
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}

int cnmf_als_prepare(double* H64, double* Ht, double* HHt, double* table, int n_features, int k,
                     double sum_to_one, void* stream) {
  return als_basis_launch(nullptr, H64, Ht, HHt, table, n_features, k, 0.0, sum_to_one, 0,
                          reinterpret_cast<hipStream_t>(stream));
}

int cnmf_als_basis_update(const double* AB, double* H64, double* Ht, double* HHt, double* table,
                          int n_features, int k, double smoothness, double sum_to_one, void* stream) {
  return als_basis_launch(AB, H64, Ht, HHt, table, n_features, k, smoothness, sum_to_one, 1,
                          reinterpret_cast<hipStream_t>(stream));
}

int cnmf_als_sample_pass(const void* X, int x_dtype, void* W, const double* Ht, const double* table,
                         double* partials, int64_t n_rows, int n_features, int k, double sum_to_one,
                         int accumulate, void* stream) {
  if (n_rows < 0) return set_err(CNMF_ERR_SHAPE, "n_rows < 0");
  if (!X || !W || !Ht || !table || (accumulate && !partials)) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (k > ALS_MAX_K) return set_err(CNMF_ERR_UNSUPPORTED, "constrained ALS supports k <= %d (got %d)", ALS_MAX_K, k);
  if (!(sum_to_one >= 0.0)) return set_err(CNMF_ERR_ARG, "sum_to_one must be >= 0");
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(W) & 15))
    return set_err(CNMF_ERR_ALIGN, "X and W must be 16-byte aligned");
  PassKernel pmain;
  size_t lmain = 0;
  int st = select_pass(x_dtype, n_features, k, &pmain, &lmain);
  if (st) return st;
  const int64_t nb = main_grid(n_rows, x_dtype, n_features, k, &pmain, &lmain);  // = partial rows
  if (nb < 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
  if (nb == 0) return CNMF_OK;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  int64_t als_rows = n_rows;
  int64_t row0 = 0, part0 = 0;
  if (accumulate && use_sl(x_dtype, n_features, k)) {
    // the sample-lane ALS pass on the full tiles (its grid = the sl grid = the first partial rows),
    // the ragged tail (< 64 rows) on one workgroup of the VALU ALS pass (partial row g)
    int64_t n_full;
    bool tail;
    const int64_t g = sl_grid(n_rows, &n_full, &tail);
    if (g < 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
    if (g > 0) {
      // its own rounds-balanced grid (2 workgroups per CU), <= g; it zeroes partial rows [ga, g)
      const int64_t ga = std::min<int64_t>(
          g, pass_grid(n_full * TS, reinterpret_cast<PassFn>(&als_pass_sl_kernel), sl::L_ALS_TOTAL));
      if (ga <= 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
      hipLaunchKernelGGL(als_pass_sl_kernel, dim3((unsigned)ga), dim3(NT), sl::L_ALS_TOTAL, hs,
                         static_cast<const float*>(X), static_cast<float*>(W), Ht, table, partials,
                         n_full, sum_to_one * sum_to_one, g);
      HIP_CHECK(hipGetLastError());
    }
    if (!tail) return CNMF_OK;
    row0 = n_full * TS;
    part0 = g;
    als_rows = n_rows - row0;
  }
  PassKernel pk;
  const int np = (n_features + k + 63) / 64;
  bool ok = false;
  switch (x_dtype) {
    case CNMF_F32: ok = pick_als_tx<float>(n_features, np, &pk); break;
    case CNMF_F64: ok = pick_als_tx<double>(n_features, np, &pk); break;
    case CNMF_BF16: ok = pick_als_tx<bf16_t>(n_features, np, &pk); break;
  }
  if (!ok) return set_err(CNMF_ERR_UNSUPPORTED, "n_features=%d too wide for the ALS pass", n_features);
  const size_t lds = pass_lds(n_features, 4, pk.sx, pk.sc, 8).total;
  if (lds > kMaxLds) return set_err(CNMF_ERR_UNSUPPORTED, "n_features=%d needs too much LDS", n_features);
  if (max_resident(pk.fn, lds) <= 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
  int F = n_features;
  int flags = CNMF_PASS_UPDATE_W | (accumulate ? CNMF_PASS_ACCUMULATE : 0);
  double d2 = sum_to_one * sum_to_one, zero = 0.0;
  const int64_t n_tiles = (als_rows + TS - 1) / TS;
  const void* Xr = static_cast<const unsigned char*>(X) + row0 * F * (int64_t)pk.sx;
  void* Wr = static_cast<unsigned char*>(W) + row0 * k * (int64_t)pk.sc;
  double* pr = partials ? partials + part0 * (int64_t)k * (F + k) : nullptr;
  const int64_t grid = row0 > 0 ? 1 : nb;
  void* args[] = {(void*)&Xr, &Wr, (void*)&Ht, (void*)&table, &pr, &als_rows, &F, &k, &d2, &zero, &flags, (void*)&n_tiles};
  HIP_CHECK(hipLaunchKernel(pk.fn, dim3((unsigned)grid), dim3(NT), args, lds, hs));
  return CNMF_OK;
}

int cnmf_reduce_update(const double* partials, int64_t n_parts, double* stage, uint32_t* counter,
                       double* AB, double* H64, double* Ht, double* HHt, int n_features, int k,
                       double l1_H, double l2_H, double* stats, void* stream) {
  int st = check_update_args(H64, Ht, HHt, n_features, k);
  if (st) return st;
  UpdateArgs ua{H64, Ht, HHt, n_features, k, padded_k(k), l1_H, l2_H, stats};
  if (ua.KP >= 8) {
    // k > 4: the reduction alone (small registers, full occupancy), then the matrix-core basis
    // update: for KP = 16 spread over the 16-feature blocks of H (basis_update_split_kernel, the
    // stage buffer free again as its scratch), else its own single-workgroup launch
    st = launch_reduce(partials, n_parts, k * (n_features + k), stage, counter, AB, 0, ua,
                       reinterpret_cast<hipStream_t>(stream));
    if (st) return st;
    if (ua.KP == 16 && !stats && n_features <= 320 &&
        (int64_t)NSLICE * k * (n_features + k) >= 256 * ((n_features + 15) / 16)) {
      hipLaunchKernelGGL(basis_update_split_kernel, dim3((unsigned)((n_features + 15) / 16)), dim3(64), 0,
                         reinterpret_cast<hipStream_t>(stream), AB, H64, Ht, HHt, n_features, k, l1_H, l2_H, stage,
                         counter + CNT_UPD);
      HIP_CHECK(hipGetLastError());
      return CNMF_OK;
    }
    return cnmf_basis_update(AB, H64, Ht, HHt, n_features, k, l1_H, l2_H, 1, stats, stream);
  }
  return launch_reduce(partials, n_parts, k * (n_features + k), stage, counter, AB, 1, ua,
                       reinterpret_cast<hipStream_t>(stream));
}

#ifdef CNMF_STAMPS
// timeline of the last persistent launch: out = [TL_IT*TL_WG*2 | TL_IT | TL_WG] u64
int cnmf_debug_timeline(unsigned long long* host_out) {
  HIP_CHECK(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_tl), sizeof(unsigned long long) * TL_IT * TL_WG * 2));
  HIP_CHECK(hipMemcpyFromSymbol(host_out + TL_IT * TL_WG * 2, HIP_SYMBOL(g_tl_pub), sizeof(unsigned long long) * TL_IT));
  HIP_CHECK(hipMemcpyFromSymbol(host_out + TL_IT * TL_WG * 2 + TL_IT, HIP_SYMBOL(g_tl_start), sizeof(unsigned long long) * TL_WG));
  HIP_CHECK(hipMemcpyFromSymbol(host_out + TL_IT * TL_WG * 2 + TL_IT + TL_WG, HIP_SYMBOL(g_tl_hw), sizeof(unsigned int) * TL_WG * 2));
  return CNMF_OK;
}
int cnmf_debug_hstep(unsigned long long* host_out) {  // [64 calls][4 rows][BPP iterations, cycles]
  HIP_CHECK(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_hs), sizeof(unsigned long long) * 64 * 4 * 2));
  return CNMF_OK;
}
int cnmf_debug_hstep_phases(unsigned long long* host_out) {  // [64 calls][4 rows][4 phases] cycles
  HIP_CHECK(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_hsp), sizeof(unsigned long long) * 64 * 4 * 4));
  return CNMF_OK;
}
int cnmf_debug_resume_phases(unsigned long long* host_out, int reset) {  // [16]: g_ph (PH)
  HIP_CHECK(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_ph), sizeof(unsigned long long) * 16));
  if (reset) {
    unsigned long long z[16] = {0};
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_ph), z, sizeof(z)));
  }
  return CNMF_OK;
}
int cnmf_debug_levels(unsigned long long* host_out) {  // g_tl_lv, g_tl_pre, g_tl_seen, g_tl_ab (mu_iter_wt_kernel)
  HIP_CHECK(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_tl_lv), sizeof(unsigned long long) * TL_IT * (TL_LVG + 1) * 2));
  HIP_CHECK(hipMemcpyFromSymbol(host_out + TL_IT * (TL_LVG + 1) * 2, HIP_SYMBOL(g_tl_pre),
                                sizeof(unsigned long long) * TL_IT * TL_WG));
  HIP_CHECK(hipMemcpyFromSymbol(host_out + TL_IT * (TL_LVG + 1) * 2 + TL_IT * TL_WG, HIP_SYMBOL(g_tl_seen),
                                sizeof(unsigned long long) * TL_IT * TL_WG));
  HIP_CHECK(hipMemcpyFromSymbol(host_out + TL_IT * (TL_LVG + 1) * 2 + 2 * TL_IT * TL_WG, HIP_SYMBOL(g_tl_ab),
                                sizeof(unsigned long long) * TL_IT * TL_WG));
  HIP_CHECK(hipMemcpyFromSymbol(host_out + TL_IT * (TL_LVG + 1) * 2 + 3 * TL_IT * TL_WG, HIP_SYMBOL(g_tl_upd),
                                sizeof(unsigned long long) * TL_IT * TL_WG));
  return CNMF_OK;
}
int cnmf_debug_xtimeline(unsigned long long* host_out) {
  HIP_CHECK(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_tl_x), sizeof(unsigned long long) * TL_IT * 4));
  return CNMF_OK;
}
int cnmf_debug_eoi(unsigned long long* host_out, int reset) {  // [16]: persistent bfw end-of-iteration phases
  HIP_CHECK(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_eoi), sizeof(unsigned long long) * 16));
  if (reset) {
    unsigned long long z[16] = {0};
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_eoi), z, sizeof(z)));
  }
  return CNMF_OK;
}
int cnmf_debug_stamps(unsigned long long* host_out, int reset) {
  HIP_CHECK(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16));
  if (reset) {
    unsigned long long z[16] = {0};
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)));
  }
  return CNMF_OK;
}
#endif

#ifdef CNMF_DIAG
int cnmf_hbm_probe(const void* buf, int64_t bytes, double* out, int n_blocks, void* stream) {
  if (!buf || !out || bytes < 16 || n_blocks < 1)
    return set_err(CNMF_ERR_ARG, "invalid hbm probe arguments");
  if (reinterpret_cast<uintptr_t>(buf) & 15) return set_err(CNMF_ERR_ALIGN, "buf must be 16-byte aligned");
  hipLaunchKernelGGL(hbm_probe_kernel, dim3(n_blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const u32x4*>(buf),
                     bytes / 16, out);
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}
#endif

// The persistent path serves fp32 X at F = 81, k = 4 with whole tiles and >= 3 tiles per workgroup
// (CNMF_PERSIST=0 disables it for A/B timing).  Returns its grid, 0 when not eligible, < 0 on error.
static bool g_no_persist = diag_env("CNMF_PERSIST") && strcmp(diag_env("CNMF_PERSIST"), "0") == 0;
// prefetch depth of the persistent kernel (CNMF_PERSIST_PD=1|2); CNMF_WRES=0 keeps W streaming
static int g_persist_pd = (diag_env("CNMF_PERSIST_PD") && atoi(diag_env("CNMF_PERSIST_PD")) == 1) ? 1 : 2;
static bool g_no_wres = diag_env("CNMF_WRES") && strcmp(diag_env("CNMF_WRES"), "0") == 0;
// The round-1 workgroup-tile kernel (mu_iter_sl_kernel: layouts 1 pairs, 2 teams, 3 floating tiles,
// DESIGN §3.0b) is instantiated in the diagnostic build only: the wave tiles (layout 4) won on every
// box, and layout 3 is not bit-repeatable (housekeeping).  In the product its launch
// functions are null and persist_grid() is 0, so every persistent launch is a wave-tile one.
#ifndef CNMF_DIAG
static PassFn persist_fn(bool = false, bool = false) { return nullptr; }
#else
static PassFn persist_fn(bool wres = false, bool multi = false) {
  if (multi)  // the multi-GPU launch: PD = 2 only
    return wres ? reinterpret_cast<PassFn>(&mu_iter_sl_kernel<2, true, true>)
                : reinterpret_cast<PassFn>(&mu_iter_sl_kernel<2, false, true>);
  if (g_persist_pd == 1)
    return wres ? reinterpret_cast<PassFn>(&mu_iter_sl_kernel<1, true>) : reinterpret_cast<PassFn>(&mu_iter_sl_kernel<1, false>);
  return wres ? reinterpret_cast<PassFn>(&mu_iter_sl_kernel<2, true>) : reinterpret_cast<PassFn>(&mu_iter_sl_kernel<2, false>);
}
#endif

static int64_t persist_grid(int64_t n_rows, int x_dtype, int F, int k, bool multi = false) {
  if (!persist_fn(false, multi)) return 0;  // the product build: wave tiles only
  if (g_no_persist || !use_sl(x_dtype, F, k) || n_rows % TS != 0) return 0;
  const int64_t n_tiles = n_rows / TS;
  const int min_tiles = g_persist_pd + 2;  // per workgroup (the W re-read hazard, see the kernel)
  if (n_tiles < min_tiles) return 0;
  const int64_t maxb = max_resident(persist_fn(false, multi), sl::L_PTOTAL);
  if (maxb <= 0) return -1;
  int64_t n_full;
  bool tail;
  const int64_t rows_cap = sl_grid(n_rows, &n_full, &tail);  // = cnmf_pass_blocks: partial rows
  if (rows_cap <= 0) return rows_cap < 0 ? -1 : 0;
  int64_t G = std::min<int64_t>({maxb, rows_cap, n_tiles / min_tiles, (int64_t)sl::GROUP * sl::MAX_GROUPS});
  const int64_t rounds = (n_tiles + G - 1) / G;
  return (n_tiles + rounds - 1) / rounds;  // <= G, so every workgroup still owns >= min_tiles
}

// LDS of the W-resident variant for this grid, or 0 when it would lower the residency
static size_t persist_wres_lds(int64_t n_rows, int64_t G, bool multi = false) {
  if (g_no_wres || G <= 0) return 0;
  const int64_t nbt_max = (n_rows / TS + G - 1) / G;
  const size_t lds = (size_t)sl::L_PTOTAL + (size_t)nbt_max * sl::WB;
  if (lds > kMaxLds) return 0;
  const int64_t base = max_resident(persist_fn(false, multi), sl::L_PTOTAL);
  const int64_t with = max_resident(persist_fn(true, multi), lds);
  return (with > 0 && with >= base) ? lds : 0;
}

// ---- layouts of the persistent MU launch (the `layout` argument of cnmf_mu_iterations /
// cnmf_mu_iterations_multi / cnmf_mu_shard_step / cnmf_persist_describe; chosen per plan, never
// process-wide): 4 = barrier-free wave tiles (mu_iter_wt_kernel, the default), 1 = pairs of 4-wave
// workgroups per CU, 2 = one 8-wave two-team workgroup per CU, 3 = pairs with floating tiles.  Which
// of 4 / 1 / 2 is fastest has differed between boxes, so MUPlan.tune() times them and keeps the
// fastest for its plan.  0 = the default (4; CNMF_PERSIST_VARIANT / CNMF_TEAMS in the diagnostic build).
static int default_layout() {
#ifndef CNMF_DIAG
  return 4;
#endif
  const char* v = diag_env("CNMF_PERSIST_VARIANT");
  if (v && atoi(v) >= 1 && atoi(v) <= 4) return atoi(v);
  return (diag_env("CNMF_TEAMS") && strcmp(diag_env("CNMF_TEAMS"), "2") == 0) ? 2 : 4;
}
static int resolve_layout(int layout) {
  if (layout == 0) return default_layout();
#ifdef CNMF_DIAG
  return (layout >= 1 && layout <= 6) ? layout : -1;
#else
  return (layout == 4 || layout == 6) ? layout : -1;
#endif
}
#define RESOLVE_LAYOUT(var)                                                                                  \
  do {                                                                                                      \
    var = resolve_layout(var);                                                                              \
    if (var < 0)                                                                                            \
      return set_err(CNMF_ERR_ARG, "layout must be 0 (default), 4 (wave tiles) or 6 (cfg4 persistent); "   \
                     "1-3 and 5 (k = 8 wave tiles on the matrix cores) are in the diagnostic build only");  \
  } while (0)
static PassFn persist_teams_fn(bool multi) {
#ifndef CNMF_DIAG
  (void)multi;
  return nullptr;
#else
  return multi ? reinterpret_cast<PassFn>(&mu_iter_sl_kernel<2, true, true, 2>)
               : reinterpret_cast<PassFn>(&mu_iter_sl_kernel<2, true, false, 2>);
#endif
}

// ---- variant 3: pairs with floating tiles (mu_iter_sl_kernel<2, true, MULTI, 1, true>): each
// workgroup keeps floor(frac · n_tiles / G) tiles resident (frac = CNMF_DYN_FRAC, default 0.8), the
// rest are drawn from a pool every iteration.  Returns the static tiles per workgroup (0: not
// eligible) and the LDS bytes.
// the resident fraction of layout 3 (CNMF_DYN_FRAC in the diagnostic build)
static double dyn_frac() {
  const char* v = diag_env("CNMF_DYN_FRAC");
  const double fr = v ? atof(v) : 0.8;
  return fr > 0.0 && fr <= 1.0 ? fr : 0.8;
}
static bool g_dyn_multi = diag_env("CNMF_DYN_MULTI") && strcmp(diag_env("CNMF_DYN_MULTI"), "1") == 0;
static PassFn persist_dyn_fn(bool multi) {
#ifndef CNMF_DIAG
  (void)multi;
  return nullptr;
#else
  return multi ? reinterpret_cast<PassFn>(&mu_iter_sl_kernel<2, true, true, 1, true>)
               : reinterpret_cast<PassFn>(&mu_iter_sl_kernel<2, true, false, 1, true>);
#endif
}
static int persist_dyn_static(int64_t n_tiles, int64_t G, bool multi, int layout, size_t* lds_out) {
  if (layout != 3 || g_no_wres || g_persist_pd != 2 || G <= 0) return 0;
  if (multi && !g_dyn_multi) return 0;  // the multi-GPU launch keeps layout 1 unless CNMF_DYN_MULTI=1
  const double frac = dyn_frac();
  const int64_t S = (int64_t)(frac * (double)n_tiles / (double)G);
  if (S < 4 || S * G > n_tiles) return 0;  // >= PD + 2 static tiles (no draw crosses an iteration)
  const size_t lds = (size_t)sl::L_PTOTAL + (size_t)S * sl::WB;
  if (lds > kMaxLds) return 0;
  if (!persist_dyn_fn(multi) || max_resident(persist_dyn_fn(multi), lds) < G) return 0;  // the whole grid co-resident
  *lds_out = lds;
  return (int)S;
}

// workgroups (0: not eligible) and LDS bytes of a two-team launch over n_tiles (persist_grid > 0)
static int64_t persist_teams_grid(int64_t n_tiles, bool multi, int layout, size_t* lds_out) {
  if (layout != 2 || g_no_wres || g_persist_pd != 2) return 0;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  const int64_t G = std::min<int64_t>({(int64_t)ncu, n_tiles / (2 * (2 + 2)), (int64_t)sl::GROUP * sl::MAX_GROUPS});
  if (G < 1) return 0;
  const int64_t nbt_max = (n_tiles + 2 * G - 1) / (2 * G);
  const size_t lds = 2 * ((size_t)sl::L_PTOTAL + (size_t)nbt_max * sl::WB);
  if (lds > kMaxLds) return 0;
  const PassFn fn = persist_teams_fn(multi);
  if (!fn) return 0;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return 0;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 2 * NT, lds) != hipSuccess) return 0;
  if (per_cu < 1) return 0;  // the whole grid must be co-resident: one workgroup per CU
  *lds_out = lds;
  return G;
}

// ---- variant 4: barrier-free wave tiles (mu_iter_wt_kernel<K, WRES, PD, MULTI>: one 4-wave
// workgroup per CU, each wave on its own tiles; fp32 X, F = 81, k = 4 (16-sample tiles) or k = 8
// (8-sample tiles); W resident in LDS when the grid's share fits, else streamed with X).
// CNMF_WT_PD = prefetch depth 2..4 of the k = 4 W-resident single-GPU kernel, 3..5 of the k = 8
// streamed-W one (default 3).
static int wt_pd(int k, bool wres, bool multi) {
  const char* v = diag_env("CNMF_WT_PD");
  const int pd = v ? atoi(v) : 3;
  if (k == 4 && wres && !multi && pd >= 2 && pd <= 4) return pd;
  if (k == 8 && !wres && !multi && pd >= 3 && pd <= 5) return pd;
  return 3;
}
extern "C++" {
template <int KK, bool WRES>
static PassFn wt_fn_k(int pd, bool multi, bool tol) {
  if (tol)  // the device tolerance test: PD = 3
    return multi ? reinterpret_cast<PassFn>(&mu_iter_wt_kernel<KK, WRES, 3, true, true>)
                 : reinterpret_cast<PassFn>(&mu_iter_wt_kernel<KK, WRES, 3, false, true>);
  if (multi) return reinterpret_cast<PassFn>(&mu_iter_wt_kernel<KK, WRES, 3, true>);
#ifdef CNMF_DIAG  // the prefetch-depth sweeps (CNMF_WT_PD): diagnostic build only
  if (KK == 4 && WRES && pd == 2) return reinterpret_cast<PassFn>(&mu_iter_wt_kernel<4, true, 2, false>);
  if (KK == 4 && WRES && pd == 4) return reinterpret_cast<PassFn>(&mu_iter_wt_kernel<4, true, 4, false>);
  if (KK == 8 && !WRES && pd == 4) return reinterpret_cast<PassFn>(&mu_iter_wt_kernel<8, false, 4, false>);
  if (KK == 8 && !WRES && pd == 5) return reinterpret_cast<PassFn>(&mu_iter_wt_kernel<8, false, 5, false>);
#else
  (void)pd;
#endif
  return reinterpret_cast<PassFn>(&mu_iter_wt_kernel<KK, WRES, 3, false>);
}
}
// the k = 8 matrix-core wave tiles (layout 5): slower than the VALU wave tiles on every box measured
// (DESIGN §3.0), so since round 6 they exist in the diagnostic build only; the
// product refuses layout 5 with CNMF_ERR_ARG
static PassFn mf8_fn(bool wres, bool multi, bool tol) {
#ifndef CNMF_DIAG
  (void)wres; (void)multi; (void)tol;
  return nullptr;
#else
  if (wres)
    return tol ? (multi ? reinterpret_cast<PassFn>(&mu_iter_mf8_kernel<true, 3, true, true>)
                        : reinterpret_cast<PassFn>(&mu_iter_mf8_kernel<true, 3, false, true>))
               : (multi ? reinterpret_cast<PassFn>(&mu_iter_mf8_kernel<true, 3, true, false>)
                        : reinterpret_cast<PassFn>(&mu_iter_mf8_kernel<true, 3, false, false>));
  return tol ? (multi ? reinterpret_cast<PassFn>(&mu_iter_mf8_kernel<false, 3, true, true>)
                      : reinterpret_cast<PassFn>(&mu_iter_mf8_kernel<false, 3, false, true>))
             : (multi ? reinterpret_cast<PassFn>(&mu_iter_mf8_kernel<false, 3, true, false>)
                      : reinterpret_cast<PassFn>(&mu_iter_mf8_kernel<false, 3, false, false>));
#endif
}
static PassFn wt_fn(int k, bool wres, bool multi, bool tol = false) {
  const int pd = tol ? 3 : wt_pd(k, wres, multi);
  if (k == 4) return wres ? wt_fn_k<4, true>(pd, multi, tol) : wt_fn_k<4, false>(pd, multi, tol);
  return wres ? wt_fn_k<8, true>(pd, multi, tol) : wt_fn_k<8, false>(pd, multi, tol);
}
static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus[dev] = 0;
  return cus[dev];
}
struct WtLaunch {
  PassFn fn;
  int64_t G, n_tiles;
  size_t lds;
  bool mf;       // k = 8 on the matrix cores (mu_iter_mf8_kernel)
  int nres = 0;  // W streamed: the first nres tiles of every wave resident in the LDS left over
  bool wres = false;  // W resident (every tile)
};
// the wave-tile launch for this shape, or false (not eligible: another kernel serves it).  k = 4
// follows the layout switch (variant 4, the default); k = 8 has no other persistent layout.
static bool wt_plan(int64_t n_rows, int x_dtype, int F, int k, bool multi, int layout, WtLaunch* out,
                    bool tol = false) {
  if (x_dtype != CNMF_F32 || F != wt::F || (k != 4 && k != 8) || n_rows <= 0) return false;
  if (k == 4 && layout != 4) return false;
  if (k == 8 && layout != 4 && layout != 5) return false;
  // k = 8, layout 4: the VALU wave tiles (8-sample tiles); layout 5 (rows a multiple of 16): the
  // matrix-core wave tiles (16-sample tiles; slower than layout 4 on the MI355X measured)
  const bool mf = k == 8 && layout == 5 && n_rows % 16 == 0;
  const int tsw = mf ? 16 : 64 / k, wbw = tsw * k * 4;
  if (n_rows % tsw != 0) return false;
  const size_t l_wres = mf ? (size_t)wt::GeoMF8::L_WRES
                           : (k == 4 ? (size_t)wt::Geo<4>::L_WRES : (size_t)wt::Geo<8>::L_WRES);
  const int ncu = device_cus();
  const int64_t n_tiles = n_rows / tsw;
  for (int wres = 1; wres >= 0; --wres) {
    const int pd = tol ? 3 : wt_pd(k, wres != 0, multi);
    // tiles per wave: > PD (the first prefetches), >= 2·PD + 1 when W is streamed (re-load hazard)
    const int min_nbt = wres ? pd + 1 : 2 * pd + 1;
    int64_t G = std::min<int64_t>({(int64_t)ncu, n_tiles / (wt::NWV * min_nbt), (int64_t)sl::GROUP * sl::MAX_GROUPS});
    if (const char* mg = diag_env("CNMF_WT_MAXG"))  // diagnostic: fewer, fuller waves (strong-scaling shards)
      if (atoi(mg) > 0) G = std::min<int64_t>(G, atoi(mg));
    if (G < 1) continue;
    const int64_t nbt_max = (n_tiles + wt::NWV * G - 1) / (wt::NWV * G);
    // W resident: the four waves' W tiles; TOL (the wave-tile kernel) a second copy: the snapshot of
    // the checked state
    size_t lds = l_wres + (wres ? (size_t)wt::NWV * nbt_max * wbw * (tol && !mf ? 2 : 1) : 0);
    if (lds > kMaxLds) continue;
    // W streamed (the VALU wave tiles): as many of each wave's tiles W-resident as the LDS holds —
    // their W neither read nor written through HBM in the iterations (cfg3's shard: ~78 % of its W
    // traffic).  CNMF_WT_NRES (diagnostic) caps it; 0 streams every tile.
    int nres = 0;
    if (!wres && !mf) {
      int64_t cap = (int64_t)((kMaxLds - lds) / ((size_t)wt::NWV * wbw));
      if (const char* nr = diag_env("CNMF_WT_NRES")) cap = std::min<int64_t>(cap, atoi(nr));
      nres = (int)std::max<int64_t>(0, std::min<int64_t>(cap, nbt_max));
      lds += (size_t)wt::NWV * nres * wbw;
    }
    const PassFn fn = mf ? mf8_fn(wres != 0, multi, tol) : wt_fn(k, wres != 0, multi, tol);
    if (max_resident(fn, lds) < G) continue;  // the whole grid co-resident (cached query)
    *out = WtLaunch{fn, G, n_tiles, lds, mf, nres, wres != 0};
    return true;
  }
  return false;
}
// the weighted wave-tile launch for this shape, or false (not served: the per-iteration pass)
struct WwLaunch {
  int64_t G, n_tiles;
  size_t lds;
};
static bool ww_plan(int64_t n_rows, int F, int k, WwLaunch* out, bool multi = false) {
  constexpr int PD = 2;
  if (F != wt::F || k != ww::K || n_rows <= 0 || n_rows % ww::TSW != 0) return false;
  if (diag_env("CNMF_WMU_PERSIST") && atoi(diag_env("CNMF_WMU_PERSIST")) == 0) return false;
  const int64_t n_tiles = n_rows / ww::TSW;
  const int64_t G = std::min<int64_t>({(int64_t)device_cus(), n_tiles / (wt::NWV * (PD + 1)),
                                       (int64_t)sl::GROUP * sl::MAX_GROUPS});
  if (G < 1) return false;
  const int64_t nbt_max = (n_tiles + wt::NWV * G - 1) / (wt::NWV * G);
  const size_t lds = (size_t)ww::L_WRES + (size_t)wt::NWV * nbt_max * wt::Geo<4>::WBW;
  if (lds > kMaxLds) return false;  // W does not fit in LDS: the per-iteration pass serves it
  const PassFn fn = multi ? reinterpret_cast<PassFn>(&wmu_iter_wt_kernel<PD, true>)
                          : reinterpret_cast<PassFn>(&wmu_iter_wt_kernel<PD>);
  if (max_resident(fn, lds) < G) return false;
  *out = WwLaunch{G, n_tiles, lds};
  return true;
}

// the persistent constrained-ALS launch for this shape, or false (the per-iteration launches serve it)
struct WaLaunch {
  int64_t G, n_tiles;
  size_t lds;
};
// The persistent ALS kernel: the W-step on the matrix cores (MX), two workgroups per CU (two waves
// per SIMD hide the MFMA, fp64 and LDS latencies, at 256 registers per lane and PD = 2) and the
// issue-priority ladder (2 steps per band).  Same-box A/B (profiles/r04/als_mx/): the VALU W-step
// 122.8 us per iteration, MX 107.7, + the ladder 105, + the Jacobi H-step 101.5, + the identity-block
// rotations and the LDS exchange of the best mask 97.3.
// (diagnostic build, CNMF_ALS_OCC: 7 the product; 2 the VALU W-step at two workgroups per CU,
// 1 one per CU, 3 one per CU with Hᵀ in VGPRs (HREG), 4 two per CU with phase 1 alone on the matrix
// cores (MF), 5 one per CU with MF, 6 MF with its B operand from LDS (MFL), 8 MX at one per CU;
// CNMF_ALS_PRIO the ladder's band, 0 = off)
static int wa_variant() {
  static const int v = diag_env("CNMF_ALS_OCC") ? atoi(diag_env("CNMF_ALS_OCC")) : 7;
  return (v >= 1 && v <= 8) ? v : 7;
}
static int wa_occ() {
  const int v = wa_variant();
  return (v == 2 || v == 4 || v == 6 || v == 7) ? 2 : 1;
}
static int wa_pd() { return wa_occ() == 1 ? 3 : 2; }  // X tiles in flight per wave
static PassFn wa_fn(bool multi = false, bool tol = false) {
  if (tol)  // the device tolerance test: the product kernel's TOL form (two workgroups per CU, PD = 2)
    return multi ? reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2, true, false, false, false, true, true>)
                 : reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2, false, false, false, false, true, true>);
#ifdef CNMF_DIAG
  if (wa_variant() == 1)
    return multi ? reinterpret_cast<PassFn>(&als_iter_wt_kernel<3, 1, true>)
                 : reinterpret_cast<PassFn>(&als_iter_wt_kernel<3, 1>);
  if (wa_variant() == 3)
    return multi ? reinterpret_cast<PassFn>(&als_iter_wt_kernel<3, 1, true, true>)
                 : reinterpret_cast<PassFn>(&als_iter_wt_kernel<3, 1, false, true>);
  if (wa_variant() == 4)
    return multi ? reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2, true, false, true>)
                 : reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2, false, false, true>);
  if (wa_variant() == 5)
    return multi ? reinterpret_cast<PassFn>(&als_iter_wt_kernel<3, 1, true, false, true>)
                 : reinterpret_cast<PassFn>(&als_iter_wt_kernel<3, 1, false, false, true>);
  if (wa_variant() == 6)
    return multi ? reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2, true, false, true, true>)
                 : reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2, false, false, true, true>);
  if (wa_variant() == 2)
    return multi ? reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2, true>)
                 : reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2>);
  if (wa_variant() == 8)
    return multi ? reinterpret_cast<PassFn>(&als_iter_wt_kernel<3, 1, true, false, false, false, true>)
                 : reinterpret_cast<PassFn>(&als_iter_wt_kernel<3, 1, false, false, false, false, true>);
#endif
  return multi ? reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2, true, false, false, false, true>)
               : reinterpret_cast<PassFn>(&als_iter_wt_kernel<2, 2, false, false, false, false, true>);
}
static bool wa_plan(int64_t n_rows, int x_dtype, int F, int k, WaLaunch* out, bool multi = false,
                    bool tol = false) {
  const int PD = tol ? 2 : wa_pd();
  const int occ = tol ? 2 : wa_occ();
  if (x_dtype != CNMF_F32 || F != wt::F || k != wa::K || n_rows <= 0 || n_rows % wa::TSW != 0) return false;
  if (diag_env("CNMF_ALS_PERSIST") && atoi(diag_env("CNMF_ALS_PERSIST")) == 0) return false;
  const int64_t n_tiles = n_rows / wa::TSW;
  // tiles per wave: >= 2·PD + 1 — the TOL form re-loads W tiles (a tile's store retires before the
  // set that re-loads it is waited for, mu_iter_wt_kernel's streamed-W rule), and the plain form
  // takes the same grid so that a fit whose test never stops is bit-identical to it
  const int min_nbt = 2 * PD + 1;
  const int64_t G = std::min<int64_t>({(int64_t)device_cus() * occ, n_tiles / (wt::NWV * min_nbt),
                                       (int64_t)sl::GROUP * sl::MAX_GROUPS});
  if (G < 1) return false;
  const size_t lds = (size_t)wa::L_HS + als_lds_bytes(F, k);
  if (lds > kMaxLds) return false;
  if (max_resident(wa_fn(multi, tol), lds) < G) return false;
  *out = WaLaunch{G, n_tiles, lds};
  return true;
}

int cnmf_als_persistent(int64_t n_rows, int n_features, int k, int x_dtype) {
  WaLaunch L;
  return wa_plan(n_rows, x_dtype, n_features, k, &L) ? 1 : 0;
}

int64_t cnmf_als_persist_workgroups(int64_t n_rows, int n_features, int k, int x_dtype, int flags) {
  WaLaunch L;
  return wa_plan(n_rows, x_dtype, n_features, k, &L, (flags & 1) != 0, (flags & 2) != 0) ? L.G : 0;
}

static int als_iterations(int n_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht, double* HHt,
                          double* table, double* partials, int64_t n_parts, double* stage, uint32_t* counter,
                          double* AB, int64_t n_rows, int n_features, int k, double sum_to_one, double smoothness,
                          uint64_t* xctl, void* const* events, int n_events, void* stream,
                          double* tolctl = nullptr) {
  if (n_iter <= 0) return CNMF_OK;
  WaLaunch L;
  const bool multi = xctl != nullptr, tol = tolctl != nullptr;
  if (!wa_plan(n_rows, x_dtype, n_features, k, &L, multi, tol))
    return set_err(CNMF_ERR_UNSUPPORTED, "the persistent constrained ALS serves fp32 F=81 k=4 with rows a multiple "
                   "of 16 and >= %d tiles of 16 rows (n_rows=%lld F=%d k=%d)", wt::NWV * (2 * (tol ? 2 : wa_pd()) + 1),
                   (long long)n_rows, n_features, k);
  if (!X || !W || !H64 || !Ht || !HHt || !table || !partials || !stage || !counter || !AB)
    return set_err(CNMF_ERR_ARG, "null pointer argument");
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(W) & 15))
    return set_err(CNMF_ERR_ALIGN, "X and W must be 16-byte aligned");
  if (!(sum_to_one >= 0.0) || !(smoothness >= 0.0)) return set_err(CNMF_ERR_ARG, "smoothness and sum_to_one must be >= 0");
  if (L.G > n_parts) return set_err(CNMF_ERR_ARG, "partials hold %lld rows, the persistent grid needs %lld",
                                    (long long)n_parts, (long long)L.G);
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  AlsPersistArgs pa;
  pa.X = static_cast<const float*>(X);
  pa.W = static_cast<float*>(W);
  pa.H64 = H64;
  pa.Ht = Ht;
  pa.HHt = HHt;
  pa.table = table;
  pa.partials = partials;
  pa.groups = stage;
  pa.AB = AB;
  pa.cnt = counter;
  pa.n_tiles = L.n_tiles;
  pa.n_iter = n_iter;
  pa.n_groups = (int)((L.G + sl::GROUP - 1) / sl::GROUP);
  if (const char* gz = diag_env("CNMF_WT_GROUP"))  // diagnostic: workgroups per first-level group
    if (atoi(gz) > 0) pa.n_groups = (int)std::min<int64_t>((L.G + atoi(gz) - 1) / atoi(gz), sl::MAX_GROUPS);
  pa.delta2 = sum_to_one * sum_to_one;
  pa.lam = smoothness;
  pa.xctl = xctl;
  pa.prio = diag_env("CNMF_ALS_PRIO") ? atoi(diag_env("CNMF_ALS_PRIO")) : 2;  // steps per ladder band
  pa.tolctl = tolctl;
  void* args[] = {&pa};
  if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[0]), hs));
  HIP_CHECK(hipLaunchKernel(reinterpret_cast<const void*>(wa_fn(multi, tol)), dim3((unsigned)L.G), dim3(NT), args,
                            L.lds, hs));
  if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[1]), hs));
  // TOL: the iteration flag may still hold the last (or the stopping) iteration: cleared in stream order
  if (tol) HIP_CHECK(hipMemsetAsync(counter + CNT_FLAG, 0, sizeof(uint32_t), hs));
  return CNMF_OK;
}

int cnmf_als_fit_tol(int max_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht, double* HHt,
                     double* table, double* partials, int64_t n_parts, double* stage, uint32_t* counter,
                     double* AB, double* tolctl, int64_t n_rows, int n_features, int k, double sum_to_one,
                     double smoothness, uint64_t* xctl, void* const* events, int n_events, void* stream) {
  if (max_iter <= 0) return set_err(CNMF_ERR_ARG, "max_iter must be >= 1");
  if (!tolctl) return set_err(CNMF_ERR_ARG, "null pointer argument");
  return als_iterations(max_iter, X, x_dtype, W, H64, Ht, HHt, table, partials, n_parts, stage, counter, AB, n_rows,
                        n_features, k, sum_to_one, smoothness, xctl, events, n_events, stream, tolctl);
}

int cnmf_als_iterations(int n_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht, double* HHt,
                        double* table, double* partials, int64_t n_parts, double* stage, uint32_t* counter,
                        double* AB, int64_t n_rows, int n_features, int k, double sum_to_one, double smoothness,
                        void* const* events, int n_events, void* stream) {
  return als_iterations(n_iter, X, x_dtype, W, H64, Ht, HHt, table, partials, n_parts, stage, counter, AB, n_rows,
                        n_features, k, sum_to_one, smoothness, nullptr, events, n_events, stream);
}

int cnmf_als_iterations_multi(int n_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht,
                              double* HHt, double* table, double* partials, int64_t n_parts, double* stage,
                              uint32_t* counter, double* AB, int64_t n_rows, int n_features, int k,
                              double sum_to_one, double smoothness, uint64_t* xctl, void* const* events,
                              int n_events, void* stream) {
  if (!xctl && n_iter > 0) return set_err(CNMF_ERR_ARG, "null exchange control block");
  return als_iterations(n_iter, X, x_dtype, W, H64, Ht, HHt, table, partials, n_parts, stage, counter, AB, n_rows,
                        n_features, k, sum_to_one, smoothness, xctl, events, n_events, stream);
}

// the first reduction level through the XCD's L2 (PersistArgs::l2rows); CNMF_WT_L2ROWS in the
// diagnostic build overrides the default
static int wt_l2rows() {
  const char* v = diag_env("CNMF_WT_L2ROWS");
  return v ? (atoi(v) != 0) : 0;
}
static int launch_wt(const WtLaunch& L, int n_iter, const void* X, void* W, double* H64, double* Ht, double* HHt,
                     double* partials, double* stage, uint32_t* counter, double* AB, double l1_W, double l2_W,
                     double l1_H, double l2_H, int apply_first, int apply_last, hipStream_t s, uint64_t* xctl,
                     double* tolctl = nullptr) {
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(W) & 15))
    return set_err(CNMF_ERR_ALIGN, "X and W must be 16-byte aligned");
  PersistArgs pa;
  pa.X = static_cast<const float*>(X);
  pa.W = static_cast<float*>(W);
  pa.H64 = H64;
  pa.Ht = Ht;
  pa.HHt = HHt;
  pa.partials = partials;
  pa.groups = stage;
  pa.AB = AB;
  pa.cnt = counter;
  pa.n_tiles = L.n_tiles;
  pa.n_iter = n_iter;
  pa.n_groups = (int)((L.G + sl::GROUP - 1) / sl::GROUP);
  if (const char* gz = diag_env("CNMF_WT_GROUP"))  // diagnostic: workgroups per first-level group
    if (atoi(gz) > 0) pa.n_groups = (int)std::min<int64_t>((L.G + atoi(gz) - 1) / atoi(gz), sl::MAX_GROUPS);
  pa.n_static = L.nres;
  pa.l1W = l1_W;
  pa.l2W = l2_W;
  pa.l1H = l1_H;
  pa.l2H = l2_H;
  pa.apply_first = apply_first;
  pa.apply_last = apply_last;
  pa.xctl = xctl;
  pa.tolctl = tolctl;
  pa.l2rows = L.mf ? 0 : wt_l2rows();
  void* args[] = {&pa};
  HIP_CHECK(hipLaunchKernel(L.fn, dim3((unsigned)L.G), dim3(NT), args, L.lds, s));
  return CNMF_OK;
}

int64_t cnmf_persist_workgroups(int64_t n_rows, int n_features, int k, int x_dtype, int layout, int multi) {
  RESOLVE_LAYOUT(layout);
  WtLaunch L;
  // multi: bit 0 = the in-launch exchange form, bit 1 = the device tolerance test's (TOL) kernel
  if (wt_plan(n_rows, x_dtype, n_features, k, (multi & 1) != 0, layout, &L, (multi & 2) != 0)) return L.G;
  if (multi & 2) return 0;  // cnmf_mu_fit_tol serves the wave tiles only
  BwpLaunch B;
  if (bwp_plan(n_rows, x_dtype, n_features, k, layout, &B)) return (multi & 1) ? 0 : B.G;  // cfg4: one GPU only
  const int64_t g = persist_grid(n_rows, x_dtype, n_features, k, (multi & 1) != 0);
  return g < 0 ? set_err(CNMF_ERR_HIP, "occupancy query failed") : g;
}

int cnmf_mu_persistent(int64_t n_rows, int n_features, int k, int x_dtype) {
  WtLaunch L;
  if (wt_plan(n_rows, x_dtype, n_features, k, false, 4, &L)) return 1;
  const int64_t g = persist_grid(n_rows, x_dtype, n_features, k);
  return g < 0 ? set_err(CNMF_ERR_HIP, "occupancy query failed") : (g > 0 ? 1 : 0);
}

int cnmf_persist_describe(int64_t n_rows, int n_features, int k, int x_dtype, int layout, char* out, int len) {
  if (!out || len < 1) return set_err(CNMF_ERR_ARG, "null pointer argument");
  RESOLVE_LAYOUT(layout);
  WtLaunch L;
  if (wt_plan(n_rows, x_dtype, n_features, k, false, layout, &L)) {
    const bool wres = L.wres;
    char wdesc[96];
    if (wres) snprintf(wdesc, sizeof wdesc, "resident in LDS");
    else if (L.nres > 0) snprintf(wdesc, sizeof wdesc, "streamed with X but for %d tiles per wave resident in LDS", L.nres);
    else snprintf(wdesc, sizeof wdesc, "streamed with X");
    if (L.mf)
      snprintf(out, (size_t)len,
               "mu_iter_mf8_kernel<k=8, W %s, PD=3>: matrix-core wave tiles of 16 samples "
               "(v_mfma_f32_16x16x4_f32), one 4-wave workgroup per CU (%lld workgroups), no barrier inside "
               "an iteration",
               wdesc, (long long)L.G);
    else
      snprintf(out, (size_t)len,
               "mu_iter_wt_kernel<k=%d, W %s, PD=%d>: wave tiles of %d samples, one 4-wave workgroup per CU "
               "(%lld workgroups), no barrier inside an iteration",
               k, wdesc, wt_pd(k, wres, false), 64 / k, (long long)L.G);
    return 1;
  }
  BwpLaunch B;
  if (bwp_plan(n_rows, x_dtype, n_features, k, layout, &B)) {
    snprintf(out, (size_t)len,
             "mu_iter_bfw_kernel<k=16, F=%d>: bf16 matrix-core wave tiles, one 4-wave workgroup per CU (%lld "
             "workgroups), reduction and basis update in the launch",
             n_features, (long long)B.G);
    return 1;
  }
  const int64_t g = persist_grid(n_rows, x_dtype, n_features, k);
  if (g < 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
  if (g == 0) {
    snprintf(out, (size_t)len, "none (per-iteration launches)");
    return 0;
  }
  static const char* names[] = {"", "pairs of 4-wave workgroups per CU", "one 8-wave two-team workgroup per CU",
                                "pairs of 4-wave workgroups per CU with floating tiles"};
  const int v = layout;
  snprintf(out, (size_t)len, "mu_iter_sl_kernel: %s (%lld workgroups)", (v >= 1 && v <= 3) ? names[v] : "?",
           (long long)g);
  return 1;
}

int64_t cnmf_counter_words(void) { return CNT_WORDS; }
int cnmf_counter_err_word(void) { return CNT_ERR; }

// ---- the multi-GPU exchange buffer (one per rank, IPC-shared): [2][world][2·K·V] tagged words
// (see the MULTI block of mu_iter_sl_kernel).  Fine-grained device memory, so a peer's
// system-scope stores and loads over xGMI are coherent with this GPU's while both kernels run.
constexpr int XBUF_MAX_WORLD = 64;
static size_t xbuf_bytes(int world) {  // [2 parities][world][2·K·V] tagged 64-bit words
  return (size_t)2 * world * 2 * (wt::Geo<8>::NOUT + 8) * sizeof(uint64_t);  // the largest accumulator set (+ loss)
}

int64_t cnmf_xbuf_bytes(int world) {
  if (world < 1 || world > XBUF_MAX_WORLD) return set_err(CNMF_ERR_ARG, "world must be in [1, %d]", XBUF_MAX_WORLD);
  return (int64_t)xbuf_bytes(world);
}

int cnmf_xbuf_alloc(int world, void** dptr, void* ipc_handle) {
  if (!dptr || !ipc_handle) return set_err(CNMF_ERR_ARG, "null pointer argument");
  const int64_t bytes = cnmf_xbuf_bytes(world);
  if (bytes < 0) return (int)bytes;
  void* p = nullptr;
  HIP_CHECK(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocFinegrained));
  hipError_t e = hipMemset(p, 0, (size_t)bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(ipc_handle), p);
  if (e != hipSuccess) {
    (void)hipFree(p);
    return set_err(CNMF_ERR_HIP, "exchange buffer: %s", hipGetErrorString(e));
  }
  *dptr = p;
  return CNMF_OK;
}

int cnmf_xbuf_handle_bytes(void) { return (int)sizeof(hipIpcMemHandle_t); }

int cnmf_device_pci_bus_id(int device, char* out, int len) {
  if (!out || len < 16) return set_err(CNMF_ERR_ARG, "buffer too small");
  HIP_CHECK(hipDeviceGetPCIBusId(out, len, device));
  return CNMF_OK;
}

int cnmf_device_can_access_peer(int device, int peer) {
  int ok = 0;
  HIP_CHECK(hipDeviceCanAccessPeer(&ok, device, peer));
  return ok ? 1 : 0;
}

int cnmf_enable_peer_access(int device, int peer) {
  if (device == peer) return CNMF_OK;
  int cur = 0;
  HIP_CHECK(hipGetDevice(&cur));
  HIP_CHECK(hipSetDevice(device));
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();  // already mapped: not an error, and not left sticky
    e = hipSuccess;
  }
  const hipError_t e2 = hipSetDevice(cur);
  if (e != hipSuccess) return set_err(CNMF_ERR_HIP, "hipDeviceEnablePeerAccess(%d -> %d): %s", device, peer, hipGetErrorString(e));
  if (e2 != hipSuccess) return set_err(CNMF_ERR_HIP, "hipSetDevice: %s", hipGetErrorString(e2));
  return CNMF_OK;
}

// ---- host-resident X (out-of-core fits: cnmf_amd/outofcore.py)
int cnmf_host_register(void* ptr, int64_t bytes) {
  if (!ptr || bytes <= 0) return set_err(CNMF_ERR_ARG, "null pointer or empty range");
  const hipError_t e = hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // a refused registration is reported, not left sticky
    return set_err(CNMF_ERR_HIP, "hipHostRegister(%lld bytes): %s", (long long)bytes, hipGetErrorString(e));
  }
  return CNMF_OK;
}

int cnmf_host_unregister(void* ptr) {
  if (!ptr) return set_err(CNMF_ERR_ARG, "null pointer argument");
  HIP_CHECK(hipHostUnregister(ptr));
  return CNMF_OK;
}

int cnmf_copy_h2d_async(void* dst, const void* src, int64_t bytes, void* stream) {
  if (!dst || !src || bytes < 0) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (bytes == 0) return CNMF_OK;
  HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, reinterpret_cast<hipStream_t>(stream)));
  return CNMF_OK;
}

int cnmf_xbuf_open(const void* ipc_handle, void** dptr) {
  if (!dptr || !ipc_handle) return set_err(CNMF_ERR_ARG, "null pointer argument");
  hipIpcMemHandle_t h;
  memcpy(&h, ipc_handle, sizeof(h));
  HIP_CHECK(hipIpcOpenMemHandle(dptr, h, hipIpcMemLazyEnablePeerAccess));
  return CNMF_OK;
}

int cnmf_xbuf_close(void* dptr) {
  HIP_CHECK(hipIpcCloseMemHandle(dptr));
  return CNMF_OK;
}

int cnmf_xbuf_free(void* dptr) {
  HIP_CHECK(hipFree(dptr));
  return CNMF_OK;
}

// one plain launch of mu_iter_sl_kernel
static int launch_persistent(int64_t G, int n_iter, const void* X, void* W, double* H64, double* Ht,
                             double* HHt, double* partials, int64_t n_parts, double* stage,
                             uint32_t* counter, double* AB, int64_t n_rows, double l1_W, double l2_W,
                             double l1_H, double l2_H, int apply_first, int apply_last, hipStream_t s,
                             int layout, uint64_t* xctl = nullptr) {
  if (G > n_parts) return set_err(CNMF_ERR_ARG, "partials hold %lld rows, the persistent grid needs %lld",
                                  (long long)n_parts, (long long)G);
  PersistArgs pa;
  pa.X = static_cast<const float*>(X);
  pa.W = static_cast<float*>(W);
  pa.H64 = H64;
  pa.Ht = Ht;
  pa.HHt = HHt;
  pa.partials = partials;
  pa.groups = stage;
  pa.AB = AB;
  pa.cnt = counter;
  pa.n_tiles = n_rows / TS;
  pa.n_iter = n_iter;
  pa.n_groups = (int)((G + sl::GROUP - 1) / sl::GROUP);
  pa.n_static = 0;
  pa.l1W = l1_W;
  pa.l2W = l2_W;
  pa.l1H = l1_H;
  pa.l2H = l2_H;
  pa.apply_first = apply_first;
  pa.apply_last = apply_last;
  pa.xctl = xctl;
  pa.tolctl = nullptr;
  const bool multi = xctl != nullptr;
  void* args[] = {&pa};
  if (n_iter > 1) {
    size_t tlds = 0;
    const int64_t GT = persist_teams_grid(n_rows / TS, multi, layout, &tlds);
    if (GT > 0 && GT <= n_parts) {
      pa.n_groups = (int)((GT + sl::GROUP - 1) / sl::GROUP);
      HIP_CHECK(hipLaunchKernel(persist_teams_fn(multi), dim3((unsigned)GT), dim3(2 * NT), args, tlds, s));
      return CNMF_OK;
    }
    size_t dlds = 0;
    const int S = persist_dyn_static(n_rows / TS, G, multi, layout, &dlds);
    if (S > 0) {
      pa.n_static = S;
      HIP_CHECK(hipLaunchKernel(persist_dyn_fn(multi), dim3((unsigned)G), dim3(NT), args, dlds, s));
      return CNMF_OK;
    }
  }
  const size_t wlds = n_iter > 1 ? persist_wres_lds(n_rows, G, multi) : 0;
  // a plain launch: the grid is at most the occupancy query's co-resident capacity (persist_grid;
  // 106 SGPRs admit 6 workgroups per CU by MI355X_MICROARCH.md's residency formula, we use 2) and
  // every wait in the kernel is bounded, so a short residency ends in the error word, not a hang.
  // (hipLaunchCooperativeKernel made rocprofv3 crash at process exit and costs ~17 us per launch.)
  if (wlds)
    HIP_CHECK(hipLaunchKernel(persist_fn(true, multi), dim3((unsigned)G), dim3(NT), args, wlds, s));
  else
    HIP_CHECK(hipLaunchKernel(persist_fn(false, multi), dim3((unsigned)G), dim3(NT), args, sl::L_PTOTAL, s));
  return CNMF_OK;
}

int cnmf_mu_shard_step(const void* X, int x_dtype, void* W, double* H64, double* Ht, double* HHt,
                       double* partials, int64_t n_parts, double* stage, uint32_t* counter, double* AB,
                       int64_t n_rows, int n_features, int k, double l1_W, double l2_W, double l1_H,
                       double l2_H, int apply_first, int layout, void* stream) {
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  RESOLVE_LAYOUT(layout);
  if ((n_rows > 0 && (!X || !W)) || !H64 || !Ht || !HHt || !stage || !counter || !AB)
    return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (n_rows == 0) {  // an empty shard (world > rows): the pending update, then zeros for the all-reduce
    if (apply_first) {
      const int st = cnmf_basis_update(AB, H64, Ht, HHt, n_features, k, l1_H, l2_H, 1, nullptr, stream);
      if (st) return st;
    }
    HIP_CHECK(hipMemsetAsync(AB, 0, sizeof(double) * k * (n_features + k), hs));
    return CNMF_OK;
  }
  {  // one wave-tile launch with n_iter = 1: the multi-iteration launch's layout, so the RCCL path
     // and the in-launch exchange sum the same partials; only tickets, no waits
    WtLaunch L;
    if (partials && wt_plan(n_rows, x_dtype, n_features, k, false, layout, &L) && L.G <= n_parts)
      return launch_wt(L, 1, X, W, H64, Ht, HHt, partials, stage, counter, AB, l1_W, l2_W, l1_H, l2_H,
                       apply_first, 0, hs, nullptr);
  }
  const int64_t G = persist_grid(n_rows, x_dtype, n_features, k);
  if (G < 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
  if (G > 0) {
    // one launch of the persistent kernel with n_iter = 1: its in-launch reduction only takes
    // tickets (no workgroup ever waits), so a plain launch is safe at any residency.  The layout
    // is the multi-iteration launch's (wave tiles by default), so the RCCL path and the in-launch
    // exchange sum the same fp32 partials.
    if (!partials) return set_err(CNMF_ERR_ARG, "null pointer argument");
    if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(W) & 15))
      return set_err(CNMF_ERR_ALIGN, "X and W must be 16-byte aligned");
    if (G > n_parts) return set_err(CNMF_ERR_ARG, "partials hold too few rows");
    PersistArgs pa;
    pa.X = static_cast<const float*>(X);
    pa.W = static_cast<float*>(W);
    pa.H64 = H64;
    pa.Ht = Ht;
    pa.HHt = HHt;
    pa.partials = partials;
    pa.groups = stage;
    pa.AB = AB;
    pa.cnt = counter;
    pa.n_tiles = n_rows / TS;
    pa.n_iter = 1;
    pa.n_groups = (int)((G + sl::GROUP - 1) / sl::GROUP);
    pa.n_static = 0;
    pa.l1W = l1_W;
    pa.l2W = l2_W;
    pa.l1H = l1_H;
    pa.l2H = l2_H;
    pa.apply_first = apply_first;
    pa.apply_last = 0;
    pa.xctl = nullptr;
    pa.tolctl = nullptr;
    void* args[] = {&pa};
    HIP_CHECK(hipLaunchKernel(persist_fn(), dim3((unsigned)G), dim3(NT), args, sl::L_PTOTAL, hs));
    return CNMF_OK;
  }
  int st;
  if (apply_first) {
    st = cnmf_basis_update(AB, H64, Ht, HHt, n_features, k, l1_H, l2_H, 1, nullptr, stream);
    if (st) return st;
  }
  st = cnmf_mu_sample_pass(X, x_dtype, W, Ht, HHt, partials, n_rows, n_features, k, l1_W, l2_W,
                           CNMF_PASS_UPDATE_W | CNMF_PASS_ACCUMULATE, stream);
  if (st) return st;
  const int64_t nb = cnmf_pass_blocks(n_rows, n_features, k, x_dtype);
  if (nb < 0) return (int)nb;
  if (nb == 0) {  // no rows: this shard contributes zeros to the all-reduce
    HIP_CHECK(hipMemsetAsync(AB, 0, sizeof(double) * k * (n_features + k), hs));
    return CNMF_OK;
  }
  return cnmf_reduce_partials(partials, nb, k * (n_features + k), stage, counter, AB, stream);
}

int cnmf_mu_iterations(int n_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht,
                       double* HHt, double* partials, int64_t n_parts, double* stage,
                       uint32_t* counter, double* AB, double* stats, int64_t n_rows,
                       int n_features, int k, double l1_W, double l2_W, double l1_H, double l2_H,
                       int layout, void* const* events, int n_events, void* stream) {
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  if (n_iter <= 0) return CNMF_OK;
  RESOLVE_LAYOUT(layout);
  {
    WtLaunch L;
    if (wt_plan(n_rows, x_dtype, n_features, k, false, layout, &L) && L.G <= n_parts) {
      if (!X || !W || !H64 || !Ht || !HHt || !partials || !stage || !counter || !AB)
        return set_err(CNMF_ERR_ARG, "null pointer argument");
      if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[0]), hs));
      const int st = launch_wt(L, n_iter, X, W, H64, Ht, HHt, partials, stage, counter, AB, l1_W, l2_W, l1_H,
                               l2_H, 0, 1, hs, nullptr);
      if (st) return st;
      if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[1]), hs));
      return CNMF_OK;
    }
  }
  {  // cfg4: the bf16 wave-tile pass with the reduction and the basis update in the launch
    BwpLaunch B;
    if (bwp_plan(n_rows, x_dtype, n_features, k, layout, &B) && B.G <= n_parts) {
      if (!X || !W || !H64 || !Ht || !HHt || !partials || !counter || !AB)
        return set_err(CNMF_ERR_ARG, "null pointer argument");
      if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(W) & 15))
        return set_err(CNMF_ERR_ALIGN, "X and W must be 16-byte aligned");
      BfwArgs ba{};
      ba.X = static_cast<const bf16_t*>(X);
      ba.W = static_cast<float*>(W);
      ba.Ht = Ht;
      ba.HHt = HHt;
      ba.partials = partials;
      ba.n_rows = n_rows;
      ba.F = n_features;
      ba.k = k;
      ba.l1 = l1_W;
      ba.l2 = l2_W;
      ba.flags = CNMF_PASS_UPDATE_W | CNMF_PASS_ACCUMULATE;
      ba.n_tiles = B.n_tiles;
      ba.H64 = H64;
      ba.Ht_out = Ht;
      ba.HHt_out = HHt;
      ba.AB = AB;
      ba.cnt = counter;
      ba.n_iter = n_iter;
      ba.l1H = l1_H;
      ba.l2H = l2_H;
      void* args[] = {&ba};
      if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[0]), hs));
      HIP_CHECK(hipLaunchKernel(reinterpret_cast<const void*>(&mu_iter_bfw_kernel), dim3((unsigned)B.G), dim3(NT),
                                args, B.lds, hs));
      if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[1]), hs));
      return CNMF_OK;
    }
  }
  const int64_t G = persist_grid(n_rows, x_dtype, n_features, k);
  if (G < 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
  if (G > 0) {
    if (!X || !W || !H64 || !Ht || !HHt || !partials || !stage || !counter || !AB)
      return set_err(CNMF_ERR_ARG, "null pointer argument");
    if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(W) & 15))
      return set_err(CNMF_ERR_ALIGN, "X and W must be 16-byte aligned");
    if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[0]), hs));
    int st = launch_persistent(G, n_iter, X, W, H64, Ht, HHt, partials, n_parts, stage, counter, AB,
                               n_rows, l1_W, l2_W, l1_H, l2_H, 0, 1, hs, layout);
    if (st) return st;
    if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[1]), hs));
    return CNMF_OK;
  }
  // events: 2·n_iter around each iteration (pass + reduction + update), or (n_events == 2) around the
  // whole n iterations — no event record between the launches of a timed stretch
  const bool ev = events && n_events >= 2 * n_iter;
  const bool ev_all = events && !ev && n_events == 2;
  if (ev_all) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[0]), hs));
  for (int it = 0; it < n_iter; ++it) {  // events around the whole iteration (pass + reduction + update)
    if (ev) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[2 * it]), hs));
    int st = cnmf_mu_sample_pass(X, x_dtype, W, Ht, HHt, partials, n_rows, n_features, k, l1_W,
                                 l2_W, CNMF_PASS_UPDATE_W | CNMF_PASS_ACCUMULATE, stream);
    if (st) return st;
    st = cnmf_reduce_update(partials, n_parts, stage, counter, AB, H64, Ht, HHt, n_features, k, l1_H,
                            l2_H, stats, stream);
    if (st) return st;
    if (ev) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[2 * it + 1]), hs));
  }
  if (ev_all) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[1]), hs));
  return CNMF_OK;
}

int64_t cnmf_xctl_words(int world) {
  if (world < 1 || world > XBUF_MAX_WORLD) return set_err(CNMF_ERR_ARG, "world must be in [1, %d]", XBUF_MAX_WORLD);
  return XC_PEERS + world;
}

int cnmf_xctl_init(uint64_t* xctl, void* const* peers, int rank, int world) {
  if (!xctl || !peers) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (world < 1 || world > XBUF_MAX_WORLD || rank < 0 || rank >= world)
    return set_err(CNMF_ERR_ARG, "rank %d / world %d out of range", rank, world);
  uint64_t h[XC_PEERS + XBUF_MAX_WORLD] = {0};
  h[XC_RANK] = (uint64_t)rank;
  h[XC_WORLD] = (uint64_t)world;
  h[XC_FLAG_OFF] = 0;  // (unused: the words carry their own tags)
  h[XC_GEN] = 0;
  for (int r = 0; r < world; ++r) {
    if (!peers[r]) return set_err(CNMF_ERR_ARG, "null exchange buffer of rank %d", r);
    h[XC_PEERS + r] = reinterpret_cast<uint64_t>(peers[r]);
  }
  HIP_CHECK(hipMemcpy(xctl, h, sizeof(uint64_t) * (XC_PEERS + world), hipMemcpyHostToDevice));
  return CNMF_OK;
}

int cnmf_mu_iterations_multi(int n_iter, const void* X, int x_dtype, void* W, double* H64,
                             double* Ht, double* HHt, double* partials, int64_t n_parts,
                             double* stage, uint32_t* counter, double* AB, int64_t n_rows,
                             int n_features, int k, double l1_W, double l2_W, double l1_H,
                             double l2_H, uint64_t* xctl, int layout, void* const* events, int n_events,
                             void* stream) {
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  if (n_iter <= 0) return CNMF_OK;
  RESOLVE_LAYOUT(layout);
  {
    WtLaunch L;
    if (wt_plan(n_rows, x_dtype, n_features, k, true, layout, &L) && L.G <= n_parts) {
      if (!X || !W || !H64 || !Ht || !HHt || !partials || !stage || !counter || !AB || !xctl)
        return set_err(CNMF_ERR_ARG, "null pointer argument");
      if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[0]), hs));
      const int st = launch_wt(L, n_iter, X, W, H64, Ht, HHt, partials, stage, counter, AB, l1_W, l2_W, l1_H,
                               l2_H, 0, 1, hs, xctl);
      if (st) return st;
      if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[1]), hs));
      return CNMF_OK;
    }
  }
  const int64_t G = persist_grid(n_rows, x_dtype, n_features, k, true);
  if (G < 0) return set_err(CNMF_ERR_HIP, "occupancy query failed");
  if (G == 0) return set_err(CNMF_ERR_UNSUPPORTED, "the in-launch multi-GPU path serves the persistent shapes only");
  if (!X || !W || !H64 || !Ht || !HHt || !partials || !stage || !counter || !AB || !xctl)
    return set_err(CNMF_ERR_ARG, "null pointer argument");
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(W) & 15))
    return set_err(CNMF_ERR_ALIGN, "X and W must be 16-byte aligned");
  if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[0]), hs));
  int st = launch_persistent(G, n_iter, X, W, H64, Ht, HHt, partials, n_parts, stage, counter, AB,
                             n_rows, l1_W, l2_W, l1_H, l2_H, 0, 1, hs, layout, xctl);
  if (st) return st;
  if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[1]), hs));
  return CNMF_OK;
}


int cnmf_tolctl_doubles(int max_iter) { return max_iter < 0 ? set_err(CNMF_ERR_ARG, "max_iter < 0") : TC_ERRS + max_iter / 10 + 1; }

int cnmf_mu_fit_tol(int max_iter, const void* X, int x_dtype, void* W, double* H64,
                    double* Ht, double* HHt, double* partials, int64_t n_parts, double* stage, uint32_t* counter,
                    double* AB, double* tolctl, int64_t n_rows, int n_features, int k, double l1_W, double l2_W,
                    double l1_H, double l2_H, int layout, uint64_t* xctl, void* const* events, int n_events,
                    void* stream) {
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  RESOLVE_LAYOUT(layout);
  if (max_iter <= 0) return set_err(CNMF_ERR_ARG, "max_iter must be >= 1");
  WtLaunch L;
  if (!wt_plan(n_rows, x_dtype, n_features, k, xctl != nullptr, layout, &L, true))
    return set_err(CNMF_ERR_UNSUPPORTED, "the device tolerance test serves the wave-tile launch (fp32 X, F = 81, "
                   "k = 4 or 8, layout 4; n_rows=%lld F=%d k=%d layout=%d)", (long long)n_rows, n_features, k, layout);
  if (L.G > n_parts) return set_err(CNMF_ERR_ARG, "partials hold %lld rows, the persistent grid needs %lld",
                                    (long long)n_parts, (long long)L.G);
  if (!X || !W || !H64 || !Ht || !HHt || !partials || !stage || !counter || !AB || !tolctl)
    return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[0]), hs));
  const int st = launch_wt(L, max_iter, X, W, H64, Ht, HHt, partials, stage, counter, AB, l1_W, l2_W, l1_H, l2_H,
                           0, 1, hs, xctl, tolctl);
  if (st) return st;
  if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[1]), hs));
  // the iteration flag may still hold the last (or the stopping) iteration: cleared in stream order
  HIP_CHECK(hipMemsetAsync(counter + CNT_FLAG, 0, sizeof(uint32_t), hs));
  return CNMF_OK;
}

// ---- weighted / masked MU
int64_t cnmf_wmu_pass_blocks(int64_t n_rows, int n_features, int k) {
  if (n_rows < 0 || n_features < 1 || n_features > 512 || k < 1 || k > 8)
    return set_err(CNMF_ERR_UNSUPPORTED, "weighted MU: n_features=%d (1..512), k=%d (1..8)", n_features, k);
  const int ts = wmu_tile(n_features, k <= 4 ? 4 : 8);
  if (ts == 0) return set_err(CNMF_ERR_UNSUPPORTED, "weighted MU: no tile fits");
  const int64_t n_tiles = (n_rows + ts - 1) / ts;
  const int64_t g2 = wmu_rows(n_features, k);
  // partial rows (one per workgroup and phase-2 group), within one reduction's capacity
  const int64_t max_wg = std::min<int64_t>(kWmuMaxBlocks, (int64_t)NSLICE * 4 * RED_ROWS_PER_THREAD / g2);
  return std::min<int64_t>(n_tiles, max_wg) * g2;
}

int cnmf_wmu_sample_pass(const float* X, const float* M, float* W, const double* H64, double* partials,
                         int64_t n_parts, int64_t n_rows, int n_features, int k, int flags, void* stream) {
  const int64_t G = cnmf_wmu_pass_blocks(n_rows, n_features, k);
  if (G < 0) return (int)G;
  if (G == 0) return CNMF_OK;  // no rows (an empty shard): nothing to read or write
  if (!X || !M || !W || !H64 || !partials) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(M) & 15) ||
      (reinterpret_cast<uintptr_t>(W) & 15))
    return set_err(CNMF_ERR_ALIGN, "X, the weights and W must be 16-byte aligned");
  const int valid = CNMF_PASS_UPDATE_W | CNMF_PASS_ACCUMULATE | CNMF_PASS_LOSS;
  if ((flags & ~valid) || flags == 0 || ((flags & CNMF_PASS_LOSS) && flags != CNMF_PASS_LOSS))
    return set_err(CNMF_ERR_ARG, "invalid flags %d", flags);
  if (G > n_parts) return set_err(CNMF_ERR_ARG, "partials hold %lld rows, the pass needs %lld",
                                  (long long)n_parts, (long long)G);
  if (G == 0) return CNMF_OK;
  const int rows = wmu_rows(n_features, k);
  const int64_t grid = G / rows;
  const int KP = k <= 4 ? 4 : 8;
  const int ts = wmu_tile(n_features, KP);
  const int64_t n_tiles = (n_rows + ts - 1) / ts;
  const size_t lds = wmu_lds(n_features, KP, ts);
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const bool two = n_features > NT;
  using Fn = void (*)(const float*, const float*, float*, const double*, double*, int64_t, int, int, int, int, int64_t, int);
  Fn fn = KP == 4 ? (two ? &wmu_pass_kernel<4, 2> : &wmu_pass_kernel<4, 1>)
                  : (two ? &wmu_pass_kernel<8, 2> : &wmu_pass_kernel<8, 1>);
  hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(NT), lds, hs, X, M, W, H64, partials, n_rows, n_features, k, ts,
                     flags, n_tiles, rows);
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}

int cnmf_wmu_persistent(int64_t n_rows, int n_features, int k) {
  WwLaunch L;
  return ww_plan(n_rows, n_features, k, &L) ? 1 : 0;
}

static int wmu_iterations(int n_iter, const float* X, const float* M, float* W, double* H64, double* partials,
                          int64_t n_parts, double* stage, uint32_t* counter, double* AD, int64_t n_rows,
                          int n_features, int k, uint64_t* xctl, void* const* events, int n_events, void* stream) {
  if (n_iter <= 0) return CNMF_OK;
  WwLaunch L;
  const bool multi = xctl != nullptr;
  if (!ww_plan(n_rows, n_features, k, &L, multi))
    return set_err(CNMF_ERR_UNSUPPORTED, "the persistent weighted MU serves fp32 F=81 k=4 with rows a multiple "
                   "of 16 whose W fits in LDS (n_rows=%lld F=%d k=%d)", (long long)n_rows, n_features, k);
  if (!X || !M || !W || !H64 || !partials || !stage || !counter || !AD)
    return set_err(CNMF_ERR_ARG, "null pointer argument");
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(M) & 15) ||
      (reinterpret_cast<uintptr_t>(W) & 15))
    return set_err(CNMF_ERR_ALIGN, "X, the weights and W must be 16-byte aligned");
  if (L.G > n_parts) return set_err(CNMF_ERR_ARG, "partials hold %lld rows, the persistent grid needs %lld",
                                    (long long)n_parts, (long long)L.G);
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  WmuPersistArgs pa;
  pa.X = X;
  pa.M = M;
  pa.W = W;
  pa.H64 = H64;
  pa.partials = partials;
  pa.groups = stage;
  pa.AD = AD;
  pa.cnt = counter;
  pa.n_tiles = L.n_tiles;
  pa.n_iter = n_iter;
  pa.n_groups = (int)((L.G + sl::GROUP - 1) / sl::GROUP);
  pa.xctl = xctl;
  void* args[] = {&pa};
  const void* fn = multi ? reinterpret_cast<const void*>(&wmu_iter_wt_kernel<2, true>)
                         : reinterpret_cast<const void*>(&wmu_iter_wt_kernel<2>);
  if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[0]), hs));
  HIP_CHECK(hipLaunchKernel(fn, dim3((unsigned)L.G), dim3(NT), args, L.lds, hs));
  if (events && n_events >= 2) HIP_CHECK(hipEventRecord(reinterpret_cast<hipEvent_t>(events[1]), hs));
  return CNMF_OK;
}

int cnmf_wmu_iterations(int n_iter, const float* X, const float* M, float* W, double* H64, double* partials,
                        int64_t n_parts, double* stage, uint32_t* counter, double* AD, int64_t n_rows,
                        int n_features, int k, void* const* events, int n_events, void* stream) {
  return wmu_iterations(n_iter, X, M, W, H64, partials, n_parts, stage, counter, AD, n_rows, n_features, k,
                        nullptr, events, n_events, stream);
}

int cnmf_wmu_iterations_multi(int n_iter, const float* X, const float* M, float* W, double* H64, double* partials,
                              int64_t n_parts, double* stage, uint32_t* counter, double* AD, int64_t n_rows,
                              int n_features, int k, uint64_t* xctl, void* const* events, int n_events,
                              void* stream) {
  if (!xctl && n_iter > 0) return set_err(CNMF_ERR_ARG, "null exchange control block");
  return wmu_iterations(n_iter, X, M, W, H64, partials, n_parts, stage, counter, AD, n_rows, n_features, k, xctl,
                        events, n_events, stream);
}

int cnmf_wmu_basis_update(const double* AD, double* H64, int n_features, int k, void* stream) {
  if (!AD || !H64) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (n_features < 1 || k < 1) return set_err(CNMF_ERR_SHAPE, "invalid shape F=%d k=%d", n_features, k);
  const int kF = k * n_features;
  hipLaunchKernelGGL(wmu_basis_kernel, dim3((unsigned)std::min(64, (kF + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), AD, H64, kF);
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}

// ---- GPU NNDSVD initialisation; see ig_gram_kernel
static int ig_blocks(int64_t n_rows) {
  const int ncu = device_cus();
  const int64_t want = (n_rows + 4095) / 4096;  // >= 4096 rows (64 tiles) per workgroup
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(want, 2 * (int64_t)std::max(ncu, 1)), 1024));
}
int64_t cnmf_init_gram_rows(int64_t n_rows) { return n_rows > 0 ? ig_blocks(n_rows) : 0; }

int cnmf_init_gram(const void* X, int x_dtype, int64_t n_rows, int n_features, double* partials,
                   int64_t n_parts, void* stream) {
  if (!X || !partials) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (n_rows < 1 || n_features < 1 || n_features > ig::FP)
    return set_err(CNMF_ERR_UNSUPPORTED, "GPU init: n_features=%d (1..%d), n_rows=%lld", n_features, ig::FP, (long long)n_rows);
  const int G = ig_blocks(n_rows);
  if (G > n_parts) return set_err(CNMF_ERR_ARG, "partials hold %lld rows, the pass needs %d", (long long)n_parts, G);
  const int64_t rpb = (n_rows + G - 1) / G;
  const size_t lds = (size_t)ig::GT * ig::FP * 8;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  switch (x_dtype) {
    case CNMF_F32: hipLaunchKernelGGL(ig_gram_kernel<float>, dim3(G), dim3(256), lds, hs, static_cast<const float*>(X), n_rows, n_features, rpb, partials); break;
    case CNMF_F64: hipLaunchKernelGGL(ig_gram_kernel<double>, dim3(G), dim3(256), lds, hs, static_cast<const double*>(X), n_rows, n_features, rpb, partials); break;
    case CNMF_BF16: hipLaunchKernelGGL(ig_gram_kernel<bf16_t>, dim3(G), dim3(256), lds, hs, static_cast<const bf16_t*>(X), n_rows, n_features, rpb, partials); break;
    default: return set_err(CNMF_ERR_ARG, "x_dtype %d", x_dtype);
  }
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}

int cnmf_init_xm(const void* X, int x_dtype, int64_t n_rows, int n_features, int k, const double* M, double* U,
                 void* stream) {
  if (!X || !M || !U) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (n_rows < 1 || n_features < 1 || n_features > ig::FP || k < 1 || k > ig::KMAX)
    return set_err(CNMF_ERR_UNSUPPORTED, "GPU init: n_features=%d (1..%d), k=%d (1..%d)", n_features, ig::FP, k, ig::KMAX);
  const int ncu = device_cus();
  const int64_t n_tiles = (n_rows + ig::GT - 1) / ig::GT;
  const int G = (int)std::max<int64_t>(1, std::min<int64_t>(n_tiles, 4 * (int64_t)std::max(ncu, 1)));
  const size_t lds = (size_t)ig::FP * ig::KMAX * 8 + (size_t)ig::GT * (n_features + 1) * 8;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  switch (x_dtype) {
    case CNMF_F32: hipLaunchKernelGGL(ig_xm_kernel<float>, dim3(G), dim3(256), lds, hs, static_cast<const float*>(X), n_rows, n_features, k, M, U); break;
    case CNMF_F64: hipLaunchKernelGGL(ig_xm_kernel<double>, dim3(G), dim3(256), lds, hs, static_cast<const double*>(X), n_rows, n_features, k, M, U); break;
    case CNMF_BF16: hipLaunchKernelGGL(ig_xm_kernel<bf16_t>, dim3(G), dim3(256), lds, hs, static_cast<const bf16_t*>(X), n_rows, n_features, k, M, U); break;
    default: return set_err(CNMF_ERR_ARG, "x_dtype %d", x_dtype);
  }
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}

int64_t cnmf_init_stats_rows(int64_t n_rows) { return n_rows > 0 ? ig_blocks(n_rows) : 0; }

int cnmf_init_stats(const double* U, int64_t n_rows, int k, double* out, int64_t n_parts, void* stream) {
  if (!U || !out) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (n_rows < 1 || k < 1 || k > ig::KMAX) return set_err(CNMF_ERR_SHAPE, "invalid shape");
  const int G = ig_blocks(n_rows);
  if (G > n_parts) return set_err(CNMF_ERR_ARG, "out holds %lld rows, the pass needs %d", (long long)n_parts, G);
  const int64_t rpb = (n_rows + G - 1) / G;
  hipLaunchKernelGGL(ig_stats_kernel, dim3(G), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), U, n_rows, k, rpb, out);
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}

int cnmf_init_fill(const double* U, int64_t n_rows, int k, const double* coef, const int* part, const double* sgn,
                   double eps, double fill, void* W, int w_dtype, void* stream) {
  if (!U || !coef || !part || !sgn || !W) return set_err(CNMF_ERR_ARG, "null pointer argument");
  if (n_rows < 1 || k < 1 || k > ig::KMAX) return set_err(CNMF_ERR_SHAPE, "invalid shape");
  const int ncu = device_cus();
  const int G = (int)std::max<int64_t>(1, std::min<int64_t>((n_rows * k + 255) / 256, 8 * (int64_t)std::max(ncu, 1)));
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  if (w_dtype == CNMF_F32)
    hipLaunchKernelGGL(ig_fill_kernel<float>, dim3(G), dim3(256), 0, hs, U, n_rows, k, coef, part, sgn, eps, fill, static_cast<float*>(W));
  else if (w_dtype == CNMF_F64)
    hipLaunchKernelGGL(ig_fill_kernel<double>, dim3(G), dim3(256), 0, hs, U, n_rows, k, coef, part, sgn, eps, fill, static_cast<double*>(W));
  else
    return set_err(CNMF_ERR_ARG, "w_dtype %d", w_dtype);
  HIP_CHECK(hipGetLastError());
  return CNMF_OK;
}
}  // extern "C"

#ifdef CNMF_PD_PROBE
// diagnostic (tools/audit_wt_asm.py): the k = 8 streamed-W wave-tile kernel at a
// prefetch depth the product never launches, compiled only to inspect its ISA
namespace cnmf {
template __global__ void mu_iter_wt_kernel<8, false, CNMF_PD_PROBE, false, false>(PersistArgs);
}
#endif
