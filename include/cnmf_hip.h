/*
 * cnmf_hip.h — C ABI of libcnmf_hip.so, the MI355X (gfx950) multiplicative-update hot path.
 *
 * The reference (AI-for-Ocean-Science/cnmf v1) has no solver and no FFI: its package
 * `cnmf/__init__.py` is 0 bytes.  The arithmetic these entry points replace is the
 * Frobenius multiplicative update of scikit-learn 1.7.2 (the reference's declared dependency,
 * /root/reference/setup.py:26,30), cited below as SK:<line> = sklearn/decomposition/_nmf.py.
 * Each entry point names the SK lines it takes over; INTEGRATION.md shows the ctypes binding.
 *
 * Layout (sklearn naming, samples-major): X[N][F] row-major, W[N][k], H[k][F].
 * W has the "compute type" TC of the X dtype: fp32 for CNMF_F32 and CNMF_BF16, fp64 for CNMF_F64;
 * the per-sample update itself is evaluated in fp64 for every dtype.  All
 * basis-side state is fp64:
 *   H64[k][F]   = the basis (master copy)
 *   Ht [F][KP]  = H transposed, zero-padded to KP = cnmf_padded_k(k) columns
 *   HHt[KP][KP] = H·Hᵀ, zero-padded.
 *   AB [k][F+k] = the reduced accumulators: AB[j][f] = (WᵀX)[j][f], AB[j][F+m] = (WᵀW)[j][m].
 *
 * Conventions.  All pointers are caller-owned device pointers (no allocation in any call except
 * the one-off occupancy query); every launch is asynchronous on `stream` (a hipStream_t, NULL = the
 * default stream); entry points return 0 or a negative cnmf_status and set a thread-local
 * message readable with cnmf_last_error().  Re-entrant; no global mutable state except that
 * message and a per-device occupancy cache; the environment is not read (the diagnostic build,
 * -DCNMF_DIAG, adds A/B switches and a bandwidth probe, and is never loaded by the product).
 */
#ifndef CNMF_HIP_H
#define CNMF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum cnmf_status {
  CNMF_OK = 0,
  CNMF_ERR_ARG = -1,         /* null pointer / bad flag / bad dtype                         */
  CNMF_ERR_SHAPE = -2,       /* n_rows < 0, F < 1, k < 1                                    */
  CNMF_ERR_UNSUPPORTED = -3, /* k > 16 or a row too wide for one LDS tile                   */
  CNMF_ERR_ALIGN = -4,       /* X or W not 16-byte aligned                                  */
  CNMF_ERR_HIP = -5          /* a HIP runtime call failed (message has hipGetErrorString)   */
};

enum cnmf_dtype { CNMF_F32 = 0, CNMF_F64 = 1, CNMF_BF16 = 2 };

enum cnmf_pass_flags {
  CNMF_PASS_UPDATE_W = 1,   /* update W in place (SK:526-631)                                */
  CNMF_PASS_ACCUMULATE = 2, /* accumulate Wᵀ_newX and Wᵀ_newW_new partials (SK:639-640)      */
  CNMF_PASS_LOSS = 4        /* only: partial sums of ‖X − W·H‖² (SK:85-129), one per block   */
};

/* ABI version (major*100 + minor) and last error message of the calling thread. */
int cnmf_abi_version(void);
const char* cnmf_last_error(void);

/* KP = 4, 8 or 16: the padded component count the kernels use for k (1 <= k <= 16). */
int cnmf_padded_k(int k);

/* Number of partial rows (= workgroups) cnmf_mu_sample_pass writes for this shape on the
 * current device; size `partials` as cnmf_pass_blocks(...) * max(1, k*(F+k)) doubles.
 * Negative on error (e.g. unsupported shape or no device). */
int64_t cnmf_pass_blocks(int64_t n_rows, int n_features, int k, int x_dtype);

/* Doubles needed by the cross-block reduction stage buffer for n_out outputs. */
int64_t cnmf_stage_doubles(int n_out);

/* One fused HBM pass over the samples (replaces SK:534-629 and the N-reductions of SK:639-640):
 *   num = X·Hᵀ, den = W·HHᵀ (+l1_W) (+l2_W·W), den==0 -> float32 eps, W <- W·(num/den)
 *   and, with CNMF_PASS_ACCUMULATE, per-workgroup fp64 partials of [WᵀX | WᵀW] using the NEW W,
 *   written to partials[block][k*(F+k)].  With CNMF_PASS_LOSS alone it writes per-workgroup
 *   partials of ‖X − W·H‖² (partials[block][0]) and changes nothing.
 *   X: [n_rows][F] of x_dtype; W: [n_rows][k] of TC; Ht, HHt: fp64 as above. */
int cnmf_mu_sample_pass(const void* X, int x_dtype, void* W, const double* Ht, const double* HHt,
                        double* partials, int64_t n_rows, int n_features, int k, double l1_W,
                        double l2_W, int flags, void* stream);

/* Deterministic fp64 column sum of partials[n_parts][n_out] into out[n_out]
 * (fixed slice order; stage: cnmf_stage_doubles(n_out) doubles; counter: one zeroed uint32 that
 * the kernel leaves zeroed). */
int cnmf_reduce_partials(const double* partials, int64_t n_parts, int n_out, double* stage,
                         uint32_t* counter, double* out, void* stream);

/* The basis update on the reduced AB (replaces SK:639-726 after the reductions):
 *   den = (WᵀW)·H (+l1_H) (+l2_H·H), den==0 -> float32 eps, H <- H·(WᵀX/den)   (do_update=1)
 * then refreshes Ht and HHt from the fp64 H64.  With do_update=0 it only derives Ht/HHt from H64
 * (first iteration, transform; AB may then be NULL).  stats (may be NULL) receives
 * {<AB_A, H>, <AB_B, H·Hᵀ>} for the cheap loss ‖X‖² − 2<A,H> + <B,HHᵀ>. */
int cnmf_basis_update(const double* AB, double* H64, double* Ht, double* HHt, int n_features, int k,
                      double l1_H, double l2_H, int do_update, double* stats, void* stream);

/* cnmf_reduce_partials followed, in the same launch (last-arriving workgroup), by
 * cnmf_basis_update(do_update=1): the single-GPU iteration tail. */
int cnmf_reduce_update(const double* partials, int64_t n_parts, double* stage, uint32_t* counter,
                       double* AB, double* H64, double* Ht, double* HHt, int n_features, int k,
                       double l1_H, double l2_H, double* stats, void* stream);

/* Words of the caller-owned uint32 counter buffer (zeroed once at allocation; every launch leaves
 * it zeroed again except the error word) and the index of its error word: non-zero after a
 * persistent launch gave up waiting for a workgroup (the results of that launch are invalid). */
int64_t cnmf_counter_words(void);
int cnmf_counter_err_word(void);

/* 1 when cnmf_mu_iterations runs this shape as ONE persistent launch (fp32 X, F = 81, k = 4 or 8,
 * n_rows a multiple of 64 / k with enough tiles per wave), 0 when it launches pass + reduce per
 * iteration. */
int cnmf_mu_persistent(int64_t n_rows, int n_features, int k, int x_dtype);

/* `layout` of a persistent launch (an argument of every call that launches one; a plan keeps its
 * own: nothing is process-wide).  Results agree to fp32 rounding of the partial sums, not bit for bit:
 *   0 = default (4);
 *   4 = wave tiles: one 4-wave workgroup per CU, each wave streaming its own 16-sample (k = 4) or
 *       8-sample (k = 8) tiles with no barrier inside an iteration, W resident in LDS when it fits;
 *   6 = bf16 X, F = 289..320, k = 16, n_rows a multiple of 64 (cfg4): n iterations as ONE launch of
 *       mu_iter_bfw_kernel (the pass, the reduction and the basis update in the launch; one GPU);
 *       layout 4 is that shape's per-iteration launches;
 * MUPlan.tune() times 4 and 6 for cfg4's shape and keeps the faster for its plan; other values are
 * CNMF_ERR_ARG.  (Diagnostic build only: layouts 1-3, the round-1 workgroup-tile kernel, DESIGN
 * §3.0b; and 5, k = 8 wave tiles with both products on the matrix cores, v_mfma_f32_16x16x4_f32 —
 * slower than layout 4 on every box measured) */

/* n_iter single-GPU MU iterations with no host synchronisation: the body of SK:831-870 for tol == 0
 * stretches.  Persistent shapes: one cooperative launch that also runs the cross-block reduction
 * and the basis update in-launch (stage then holds the group rows, counter: cnmf_counter_words()).
 * Other shapes: pass + reduce_update per iteration.
 * events (may be NULL), caller-created hipEvent_t recorded on `stream` for live kernel timing:
 *   persistent: events[0] / events[1] before / after the launch (n_events >= 2);
 *   otherwise : events[2i] / events[2i+1] around iteration i: its pass, reduction and basis
 *               update (n_events >= 2*n_iter), or, n_events == 2, events[0] / events[1] around
 *               all n_iter iterations (no event record between the launches).
 * Persistent shapes: fp32 F = 81, k = 4 / 8 (mu_iter_wt_kernel), and with layout 6 bf16
 * F = 289..320, k = 16, n_rows a multiple of 64 (mu_iter_bfw_kernel, cfg4). */
int cnmf_mu_iterations(int n_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht,
                       double* HHt, double* partials, int64_t n_parts, double* stage,
                       uint32_t* counter, double* AB, double* stats, int64_t n_rows,
                       int n_features, int k, double l1_W, double l2_W, double l1_H, double l2_H,
                       int layout, void* const* events, int n_events, void* stream);

/* One MU iteration of a row shard for the multi-GPU driver (SK:831-870 with the accumulators
 * all-reduced between ranks):
 *   apply_first = 1: first the pending basis update from AB (= the all-reduced [WᵀX | WᵀW] of the
 *                    previous iteration; SK:634-728), refreshing H64 / Ht / HHt;
 *   then the W update of this shard (SK:526-631) and this shard's reduced [WᵀX | WᵀW] into AB.
 * The caller all-reduces AB (RCCL) and passes apply_first = 1 next time; cnmf_basis_update applies
 * the last pending update.  Persistent shapes run as ONE launch of the persistent kernel. */
int cnmf_mu_shard_step(const void* X, int x_dtype, void* W, double* H64, double* Ht, double* HHt,
                       double* partials, int64_t n_parts, double* stage, uint32_t* counter, double* AB,
                       int64_t n_rows, int n_features, int k, double l1_W, double l2_W, double l1_H,
                       double l2_H, int apply_first, int layout, void* stream);

/* ---- Multi-GPU with the all-reduce inside the persistent launch (persistent shapes only).
 * Each rank allocates one exchange buffer (fine-grained device memory, zeroed) and exports its IPC
 * handle (cnmf_xbuf_handle_bytes() bytes); every rank opens every peer's handle and writes the
 * pointers (its own at [rank]) into a device control block of cnmf_xctl_words(world) uint64 words
 * with cnmf_xctl_init; then
 *   cnmf_mu_iterations_multi(n, ..., xctl, ...)
 * = n iterations of SK:831-870 over the union of the shards, as ONE launch per rank: each
 * iteration's [WᵀX | WᵀW] goes to every peer over xGMI and is summed in rank order (the same AB on
 * every rank, bit for bit); the last iteration's basis update is applied in-launch like
 * cnmf_mu_iterations.  The control block also holds the exchange generation (word 3), advanced
 * on the device by every launch, so all ranks must issue the same sequence of launches.  Every wait
 * is bounded: a rank that times out sets the counter's error word and poisons its flags so that
 * every peer's launch fails too; the buffer set is then unusable (fall back to
 * cnmf_mu_shard_step + an RCCL all-reduce). */
/* The persistent launch cnmf_mu_iterations would use for this shape, as text (kernel, layout,
 * W residency, grid) into out[len]; returns 1 (persistent), 0 (per-iteration launches) or < 0. */
int cnmf_persist_describe(int64_t n_rows, int n_features, int k, int x_dtype, int layout, char* out,
                          int len);
int64_t cnmf_xbuf_bytes(int world);
int cnmf_xbuf_handle_bytes(void);
/* Peer checks before the exchange: the PCI bus id of a visible device ("dddd:bb:dd.f", len >= 16)
 * and whether `device` can map `peer`'s memory (1 / 0). */
int cnmf_device_pci_bus_id(int device, char* out, int len);
int cnmf_device_can_access_peer(int device, int peer);
/* Map `peer`'s memory into `device`'s kernels (hipDeviceEnablePeerAccess with `device` current;
 * idempotent; the current device is restored) — several devices driven from ONE process
 * (cnmf_amd.multidevice) exchange through directly mapped buffers, no IPC. */
int cnmf_enable_peer_access(int device, int peer);
/* Workgroups of the persistent launch for this shape and layout, 0 when the shape runs
 * per-iteration launches; every one is resident for the whole launch (one per CU for the wave
 * tiles), so co-running launches on one device must fit together.  multi: bit 0 = the in-launch
 * exchange form (cnmf_mu_iterations_multi), bit 1 = the launch of cnmf_mu_fit_tol (0 when the
 * device tolerance test does not serve the shape). */
int64_t cnmf_persist_workgroups(int64_t n_rows, int n_features, int k, int x_dtype, int layout, int multi);
int cnmf_xbuf_alloc(int world, void** dptr, void* ipc_handle);
int cnmf_xbuf_open(const void* ipc_handle, void** dptr);
int cnmf_xbuf_close(void* dptr);
int cnmf_xbuf_free(void* dptr);
int64_t cnmf_xctl_words(int world);
int cnmf_xctl_init(uint64_t* xctl, void* const* peers, int rank, int world);
int cnmf_mu_iterations_multi(int n_iter, const void* X, int x_dtype, void* W, double* H64,
                             double* Ht, double* HHt, double* partials, int64_t n_parts,
                             double* stage, uint32_t* counter, double* AB, int64_t n_rows,
                             int n_features, int k, double l1_W, double l2_W, double l1_H,
                             double l2_H, uint64_t* xctl, int layout, void* const* events, int n_events,
                             void* stream);

/* ---- The tolerance test on the device (SK:872-884 without a host round trip).
 * cnmf_mu_fit_tol runs up to max_iter MU iterations of the wave-tile launch (fp32 X, F = 81, k = 4
 * or 8, layout 0 / 4; xctl NULL = one GPU, else the in-launch exchange as cnmf_mu_iterations_multi)
 * as ONE launch that also evaluates ‖X − W·H‖ of the state after g iterations (g = it0, it0 + 10,
 * ...: in the pass of iteration g + 1, which already reads x and w) and stops on the device when
 * (previous − error) / error_at_init < tol — sklearn's n_iter, W and H exactly as its loop leaves
 * them.  Buffers as cnmf_mu_iterations' except: partials rows, stage and AB hold k·(F+k) + 2
 * doubles (the loss column and a pad: ABI 302, rows of whole 16-byte chunks); tolctl = cnmf_tolctl_doubles(max_iter) doubles with, set by the
 * caller: [CNMF_TC_TOL] tol (> 0), [CNMF_TC_IT0] it0 (global index of the launch's first
 * iteration; its errors go to slots g / 10), [CNMF_TC_CAP] error slots after CNMF_TC_ERRS,
 * [CNMF_TC_WSNAP] a device buffer of n_rows·k floats (bits of the pointer; used when W is streamed,
 * k = 8 past the LDS limit), and when it0 > 0 [CNMF_TC_INIT] / [CNMF_TC_PREV] from the previous
 * launch.  Out: [CNMF_TC_DONE] iterations done (global), [CNMF_TC_STOPPED] 1 if the test stopped
 * the fit, [CNMF_TC_IN_SNAP] 1 if the stopped fit's W is in the snapshot buffer (copy it to W),
 * [CNMF_TC_NERR] and the checked errors from [CNMF_TC_ERRS].  The counter's flag word is cleared
 * in stream order after the launch. */
enum cnmf_tolctl_slots {
  CNMF_TC_TOL = 0, CNMF_TC_IT0 = 1, CNMF_TC_INIT = 2, CNMF_TC_PREV = 3, CNMF_TC_DONE = 4, CNMF_TC_STOPPED = 5,
  CNMF_TC_IN_SNAP = 6, CNMF_TC_WSNAP = 7, CNMF_TC_CAP = 8, CNMF_TC_NERR = 9, CNMF_TC_ERRS = 16
};
int cnmf_tolctl_doubles(int max_iter);
int cnmf_mu_fit_tol(int max_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht, double* HHt,
                    double* partials, int64_t n_parts, double* stage, uint32_t* counter, double* AB,
                    double* tolctl, int64_t n_rows, int n_features, int k, double l1_W, double l2_W,
                    double l1_H, double l2_H, int layout, uint64_t* xctl, void* const* events, int n_events,
                    void* stream);

/* Normalisation projection (no sklearn counterpart, off unless asked for):
 *   s_j = ‖H_j‖ (norm 1 = L1, 2 = L2, 3 = max; s_j := 1 for an all-zero row),
 *   H_j <- H_j / s_j (H64, and Ht / HHt refreshed), W[:, j] <- W[:, j]·s_j, scale[j] = s_j,
 * so W·H is unchanged.  W: [n_rows][k] of w_dtype (CNMF_F32 or CNMF_F64); scale: k doubles. */
int cnmf_normalise(void* W, int w_dtype, double* H64, double* Ht, double* HHt, double* scale,
                   int64_t n_rows, int n_features, int k, int norm, void* stream);

/* ---- Constrained ALS (no sklearn counterpart — the spec and its
 * scipy-NNLS oracle are oracle/als_ref.py; DESIGN.md §Constrained ALS).  k <= 4, F <= 512.
 * table: cnmf_als_table_doubles() doubles = the W-step's passive-set inverses of
 * Q = HHᵀ + δ²11ᵀ (δ = sum_to_one), rebuilt by every basis call. */
int cnmf_als_table_doubles(void);

/* Ht / HHt / table from H64 (no update): before the first W-step. */
int cnmf_als_prepare(double* H64, double* Ht, double* HHt, double* table, int n_features, int k,
                     double sum_to_one, void* stream);

/* The W-step over all samples (one HBM pass): w_i = argmin_{w>=0} ‖x_i − Hᵀw‖² + δ²(1ᵀw − 1)²
 * exactly (passive-set enumeration on the Gram form), written to W; with accumulate, the
 * per-workgroup fp64 partials of [WᵀX | WᵀW] of the new W (rows: cnmf_pass_blocks). */
int cnmf_als_sample_pass(const void* X, int x_dtype, void* W, const double* Ht, const double* table,
                         double* partials, int64_t n_rows, int n_features, int k, double sum_to_one,
                         int accumulate, void* stream);

/* The H-step on the reduced AB = [WᵀX | WᵀW]: one Gauss-Seidel sweep of exact NNLS rows
 * h_j = argmin_{h>=0} ½hᵀ(B_jj I + λDᵀD)h − (a_j − Σ_{m≠j} B_jm h_m)ᵀh (λ = smoothness, D the
 * second difference), then Ht, HHt and the table for the next W-step. */
int cnmf_als_basis_update(const double* AB, double* H64, double* Ht, double* HHt, double* table,
                          int n_features, int k, double smoothness, double sum_to_one, void* stream);

/* n constrained-ALS iterations (W-step, [WᵀX | WᵀW], H-step) as ONE persistent launch
 * (als_iter_wt_kernel).  Served shape (cnmf_als_persistent returns 1): fp32 X, n_features = 81,
 * k = 4, n_rows a multiple of 16; else 0 and cnmf_als_iterations returns CNMF_ERR_UNSUPPORTED (run
 * cnmf_als_sample_pass + cnmf_reduce_partials + cnmf_als_basis_update per iteration).  The W-step
 * reads H64 (and derives Ht / HHt / the table itself); on return H64, Ht, HHt and table hold the
 * final basis state, W the last W-step, AB the last iteration's reduced accumulators.  Buffers as
 * cnmf_mu_iterations'; a workgroup that is never co-resident makes the launch give up and set
 * counter[cnmf_counter_err_word()] (results then invalid).  events: optional 2 recorded events. */
int cnmf_als_persistent(int64_t n_rows, int n_features, int k, int x_dtype);
int cnmf_als_iterations(int n_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht, double* HHt,
                        double* table, double* partials, int64_t n_parts, double* stage, uint32_t* counter,
                        double* AB, int64_t n_rows, int n_features, int k, double sum_to_one, double smoothness,
                        void* const* events, int n_events, void* stream);
/* The same on several GPUs, one launch per rank: each rank's reduced [WᵀX | WᵀW] is summed with the
 * other ranks' inside the launch (the in-launch exchange of cnmf_mu_iterations_multi: xctl from
 * cnmf_xctl_init over buffers from cnmf_xbuf_alloc / cnmf_xbuf_open), so every rank applies the
 * same H-step.  Every rank must issue the same sequence of launches. */
int cnmf_als_iterations_multi(int n_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht,
                              double* HHt, double* table, double* partials, int64_t n_parts, double* stage,
                              uint32_t* counter, double* AB, int64_t n_rows, int n_features, int k,
                              double sum_to_one, double smoothness, uint64_t* xctl, void* const* events,
                              int n_events, void* stream);
/* Workgroups of the persistent ALS launch for this shape (0: not served).  flags bit 0: the
 * exchange form (cnmf_als_iterations_multi); bit 1: the tolerance-test form (cnmf_als_fit_tol, which
 * needs >= 5 tiles of 16 rows per wave). */
int64_t cnmf_als_persist_workgroups(int64_t n_rows, int n_features, int k, int x_dtype, int flags);
/* A max_iter constrained-ALS fit with the tolerance test of oracle/als_ref.py (SK:872-884's rule:
 * ‖X − WH‖ every 10 iterations, stop when (previous − error) / error_at_init < tol) evaluated on the
 * device: ONE launch of the persistent kernel (replaces the host loop of `run_mu` over
 * cnmf_als_iterations + a loss pass per 10 iterations).  tolctl: cnmf_tolctl_doubles(max_iter)
 * doubles laid out as for cnmf_mu_fit_tol (CNMF_TC_*; TC_WSNAP = the address of an N x k fp32
 * snapshot buffer as a double's bits).  On a stop at g iterations: H64 / Ht / HHt / table hold the
 * basis after g iterations, the snapshot buffer holds W after g iterations (TC_IN_SNAP = 1: the
 * caller copies it to W), TC_DONE = g.  xctl: null, or the exchange block (several GPUs, every
 * rank the same max_iter and tol).  partials / stage / AB: rows of k(F + k) + 1 doubles. */
int cnmf_als_fit_tol(int max_iter, const void* X, int x_dtype, void* W, double* H64, double* Ht, double* HHt,
                     double* table, double* partials, int64_t n_parts, double* stage, uint32_t* counter,
                     double* AB, double* tolctl, int64_t n_rows, int n_features, int k, double sum_to_one,
                     double smoothness, uint64_t* xctl, void* const* events, int n_events, void* stream);


/* ---- weighted / masked MU (oracle/wmu_ref.py).  Per-element weights
 * M >= 0 (N x F fp32, same layout as X; 0 = missing):
 *   W <- W o ((M o X) H^T) / ((M o (W H)) H^T),   H <- H o (W'^T (M o X)) / (W'^T (M o (W' H)))
 * (SK:831-870 order and zero-denominator rule SK:620 / SK:706; with M = 1 exactly SK's Frobenius
 * MU, SK:526-728).  No reference interface: the reference's MU has no weights.  fp32 X / M / W,
 * H64 the fp64 master basis (k x F); 1 <= k <= 8, 1 <= F <= 512.
 * cnmf_wmu_pass_blocks: partial rows of one pass (size `partials` as that x 2kF doubles; x 1 for
 * the loss).  cnmf_wmu_sample_pass flags: UPDATE_W | ACCUMULATE (each workgroup's fp64 row
 * [W'^T(MoX) | W'^T(Mo(W'H))]) or LOSS alone (each row: sum m (x - wh)^2).  Reduce the rows with
 * cnmf_reduce_partials (n_out = 2kF, or 1), then cnmf_wmu_basis_update(AD) applies the H-step. */
int64_t cnmf_wmu_pass_blocks(int64_t n_rows, int n_features, int k);
int cnmf_wmu_sample_pass(const float* X, const float* M, float* W, const double* H64, double* partials,
                         int64_t n_parts, int64_t n_rows, int n_features, int k, int flags, void* stream);
int cnmf_wmu_basis_update(const double* AD, double* H64, int n_features, int k, void* stream);

/* n weighted MU iterations (W-step, [A | D] of the new W, H-step) as ONE persistent launch
 * (wmu_iter_wt_kernel: the in-launch reduction and H-step of cnmf_mu_iterations' wave-tile kernel).
 * Served shape (cnmf_wmu_persistent returns 1): fp32 X / M, n_features = 81, k = 4, n_rows a
 * multiple of 16 whose W fits in LDS (<= ~1.6e6 rows); else 0 and cnmf_wmu_iterations returns
 * CNMF_ERR_UNSUPPORTED (run cnmf_wmu_sample_pass + cnmf_reduce_partials + cnmf_wmu_basis_update per
 * iteration).  Buffers as cnmf_wmu_sample_pass's (partials: cnmf_wmu_pass_blocks rows of 2kF;
 * stage: cnmf_stage_doubles(2kF); counter: cnmf_counter_words(), zero and left zero); AD receives
 * the last iteration's reduced accumulators, H64 the final basis, W the final W.  A workgroup that
 * is never co-resident makes the launch give up and set counter[cnmf_counter_err_word()]: the
 * results are then invalid (the host checks the word).  events: optional 2 recorded events around
 * the launch (timing). */
int cnmf_wmu_persistent(int64_t n_rows, int n_features, int k);
int cnmf_wmu_iterations(int n_iter, const float* X, const float* M, float* W, double* H64, double* partials,
                        int64_t n_parts, double* stage, uint32_t* counter, double* AD, int64_t n_rows,
                        int n_features, int k, void* const* events, int n_events, void* stream);
/* The same on several GPUs, one launch per rank, the reduced [A | D] summed over the ranks inside the
 * launch (the exchange of cnmf_mu_iterations_multi; xctl from cnmf_xctl_init). */
int cnmf_wmu_iterations_multi(int n_iter, const float* X, const float* M, float* W, double* H64, double* partials,
                              int64_t n_parts, double* stage, uint32_t* counter, double* AD, int64_t n_rows,
                              int n_features, int k, uint64_t* xctl, void* const* events, int n_events,
                              void* stream);


/* ---- GPU NNDSVD initialisation (sklearn _initialize_nmf SK:317-373 over
 * randomized_svd, extmath.py:530-604).  The device does the passes over X; the host the F x r
 * algebra (cnmf_amd/gpu_init.py).  n_features <= 96, k <= 16.
 *
 * cnmf_init_gram: per-workgroup fp64 rows [X^T X (F*F) | column sums of X (F)] into partials
 *   (cnmf_init_gram_rows(n_rows) rows of F*F + F doubles; reduce them with cnmf_reduce_partials).
 *   Replaces the X @ Q / X.T @ Q products of _randomized_range_finder (extmath.py:287-357): only
 *   span(Q) enters the result, and span(X^T X Q) needs only X^T X.
 * cnmf_init_xm: U = X * M (n_rows x k, fp64), M: F x k fp64 (row-major) — the final U = Q @ Uhat
 *   (extmath.py:586-590) as one pass over X.
 * cnmf_init_stats: per workgroup and column j of U: {sum max(u,0)^2, sum min(u,0)^2, max |u|, the u
 *   at the first row attaining it, that row} (cnmf_init_stats_rows(n_rows) rows of 5k doubles):
 *   svd_flip's u-based signs (extmath.py:900-953) and the NNDSVD part norms (SK:344-357).
 * cnmf_init_fill: W[n][j] = coef[j] * part_j(sgn[j] * U[n][j]) (part 0: |u|, 1: max(u,0),
 *   2: |min(u,0)|), then < eps -> 0, then 0 -> fill (SK:339-369 for nndsvd / nndsvda). */
int64_t cnmf_init_gram_rows(int64_t n_rows);
int cnmf_init_gram(const void* X, int x_dtype, int64_t n_rows, int n_features, double* partials,
                   int64_t n_parts, void* stream);
int cnmf_init_xm(const void* X, int x_dtype, int64_t n_rows, int n_features, int k, const double* M,
                 double* U, void* stream);
int64_t cnmf_init_stats_rows(int64_t n_rows);
int cnmf_init_stats(const double* U, int64_t n_rows, int k, double* out, int64_t n_parts, void* stream);
int cnmf_init_fill(const double* U, int64_t n_rows, int k, const double* coef, const int* part,
                   const double* sgn, double eps, double fill, void* W, int w_dtype, void* stream);

/* ---- Host-resident X (fits whose X exceeds HBM or a memory budget,
 * cnmf_amd/outofcore.py).  The chunked fit runs cnmf_mu_shard_step per row chunk (apply_first = 0,
 * AB -> one row per chunk), cnmf_reduce_partials over the chunk rows, then cnmf_basis_update.
 * cnmf_host_register: page-lock `bytes` of host memory in place (hipHostRegister) so chunk copies
 *   from it are DMA transfers; fails (status < 0, no sticky error) for memory that cannot be
 *   locked (e.g. a read-only file mapping): stage through pinned buffers instead.
 * cnmf_copy_h2d_async: hipMemcpyAsync host -> device on `stream`. */
int cnmf_host_register(void* ptr, int64_t bytes);
int cnmf_host_unregister(void* ptr);
int cnmf_copy_h2d_async(void* dst, const void* src, int64_t bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* CNMF_HIP_H */
