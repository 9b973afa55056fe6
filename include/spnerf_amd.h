/*
 * spnerf_amd.h — C ABI of the MI355X (gfx950) SP-NeRF volumetric render path.
 *
 * Plain pointers, sizes and an opaque `void* stream` (a hipStream_t; NULL = the
 * default stream).  No torch types cross this boundary.  Every device pointer is
 * owned by the caller: the library NEVER allocates device memory — callers size
 * buffers with the *_bytes() queries below and pass them in.  Every entry point
 * is stream-ordered and returns 0 on success or a negative error code; the text
 * of the last error on the calling thread is spnerf_last_error().
 *
 * Each entry point replaces a reference interface (file:line in the reference
 * ShiningFeng/SP-NeRF tree).  The Python mirror of those interfaces lives in
 * sp-nerf_amd/ (rendering.py, spnerf.py); INTEGRATION.md shows the ctypes binding.
 */
#ifndef SPNERF_AMD_H
#define SPNERF_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ---------------------------------------------------------------------- */
#define SPNERF_OK 0
#define SPNERF_E_ARG -1       /* bad shape / flag / null pointer                         */
#define SPNERF_E_HIP -2       /* a HIP runtime call failed                               */
#define SPNERF_E_UNSUPPORTED -3

/* ---- model description: the SPNeRF construction flags (models/__init__.py:6-13,
 *      models/spnerf.py:162-271) ---------------------------------------------------------- */
typedef struct spnerf_model_cfg {
    int32_t width;        /* --fc_units W (spnerf.py:163 `feat`)                              */
    int32_t layers;       /* --fc_layers (8)                                                  */
    int32_t skip;         /* skip-connection layer (skips=[4]); -1 = none                     */
    int32_t n_freq;       /* positional-encoding frequencies (10); 0 = --mapping off          */
    int32_t sem_classes;  /* --num_sem_classes C when --sem, else 0                           */
    int32_t sem_dim;      /* C * --s_embedding_factor when --sem, else 0                      */
    int32_t beta;         /* --beta: uncertainty head on                                      */
    int32_t t_dim;        /* --t_embbeding_tau (beta only)                                    */
    int32_t dtype;        /* 0 = fp32 everywhere; 1 = bf16 MFMA trunk (fp32 encode + layer 0) */
    int32_t reserved[7];
} spnerf_model_cfg;

/* ---- on-device random draws (counter-based Philox keyed by seed, step and ray)
 * The render path's draws — stratified jitter (rendering.py:143), the guided windows'
 * uniforms (:35 via :87, :113), sample_pdf's uniforms (:35) and the sigma noise (spnerf.py:122) —
 * are generated inside the kernels that consume them when a key is passed instead of a draw
 * buffer: draw `i` of ray `r` in slot `s` = Philox4x32-10(counter = (ray0 + r, s << 16 | i,
 * step), key = seed) with state = {seed, step} read from DEVICE memory (so a captured HIP graph
 * replays with the step its caller advanced).  Uniforms take 24 bits, [0, 1) like torch's
 * float uniform; normals are Box–Muller of two of the four words.  A draw depends only on
 * (seed, step, ray0 + r, slot, i): data-parallel ranks that pass ray0 = their first global
 * ray reproduce the single-process draws bit for bit. */
typedef struct spnerf_rng {
    const int64_t* state;  /* device {seed, step}                                             */
    int64_t ray0;          /* global id of ray 0 of this call                                 */
    int32_t slot;          /* draw stream (the guided sampler uses slot and slot + 1)         */
    int32_t reserved;
} spnerf_rng;

/* mlp flags */
#define SPNERF_MLP_SAVE 1        /* keep activations for spnerf_mlp_backward (training)      */
#define SPNERF_MLP_SIGMA_ONLY 2  /* trunk + sigma head only (pass 1 of guided sampling)      */
#define SPNERF_MLP_SUN_ONLY 4    /* sigma + sun-visibility heads (solar-correction pass)     */
#define SPNERF_MLP_ACCUMULATE 8  /* backward: add into grad_flat instead of overwriting it   */
#define SPNERF_MLP_DEFER_TRUNK_WGRAD 16  /* backward: leave the trunk (and sun_v 2/4) weight gradients to
                                          * spnerf_mlp_trunk_wgrad (the workspace must stay intact) */

/* composite flags */
#define SPNERF_COMP_WEIGHTS_ONLY 1  /* weights, transparency, depth only (no rgb / sem)      */
#define SPNERF_COMP_SUN_COLUMN 2    /* with WEIGHTS_ONLY: `rgb` receives the sun-visibility column
                                     * (n_rays, n_samples) of `out` (the solar pass's sun_sc,
                                     * rendering.py:177) and the backward's g_rgb is its gradient,
                                     * written into d_out's sun column (no separate slice gradient) */

/* ---- library ---------------------------------------------------------------------------- */
const char* spnerf_last_error(void);
int32_t spnerf_abi_version(void);

/* ---- parameters: canonical order == SPNeRF.named_parameters() (spnerf.py:162-264) ------ */
int32_t spnerf_param_count(const spnerf_model_cfg* cfg);
/* name of parameter `idx` (state-dict key) and its torch shape (cols = 0 for 1-D tensors) */
int32_t spnerf_param_info(const spnerf_model_cfg* cfg, int32_t idx, char* name, int32_t name_cap,
                          int64_t* rows, int64_t* cols);
int64_t spnerf_packed_bytes(const spnerf_model_cfg* cfg);
/* Re-lays the torch parameters (device pointers, canonical order) into the kernel layout:
 * padded K, pre-transposed copies for the backward, concatenated sibling heads.
 * `packed` must be zero-filled once when allocated (padding is never written). */
int32_t spnerf_pack_params(const spnerf_model_cfg* cfg, const float* const* params, void* packed, void* stream);

/* ---- per-point network: SPNeRF.forward (spnerf.py:273-369) over the points of
 *      `n_rays` rays x `n_samples` depths, xyz = rays[:,0:3] + rays[:,dir:dir+3] * z
 *      (rendering.py:147,168,172).  out is (P, n_outputs) [rgb3, sigma, sun, sky3, (beta), sem]. */
int64_t spnerf_mlp_workspace_bytes(const spnerf_model_cfg* cfg, int64_t n_rays, int32_t n_samples, int32_t flags);
int32_t spnerf_mlp_forward(const spnerf_model_cfg* cfg, const void* packed,
                           const float* rays, int32_t ray_stride, int32_t dir_offset,
                           int64_t n_rays, int32_t n_samples, const float* z,
                           const int64_t* labels, const float* t_emb, int32_t flags,
                           void* workspace, float* out, void* stream);
/* spnerf_mlp_forward over rays [ray_begin, ray_begin + n_rays) of a workspace laid out for
 * n_rays_total rays (spnerf_mlp_workspace_bytes(cfg, n_rays_total, n_samples, flags)): rays, z,
 * labels, t_emb and out are the window's own rows; depth j of ray r is z[r * z_stride + j]
 * (z_stride 0 = n_samples).  Windows filled at different times make ONE
 * saving forward whose backward runs over all n_rays_total rays — render_rays' guided main pass
 * (rendering.py:159-170) evaluates its stratified half in pass 1 (window 0, whose sigma feeds
 * the guided windows) and only the guided half afterwards (window 1, the rays repeated), instead
 * of evaluating the stratified points twice. */
int32_t spnerf_mlp_forward_window(const spnerf_model_cfg* cfg, const void* packed,
                                  const float* rays, int32_t ray_stride, int32_t dir_offset,
                                  int64_t n_rays_total, int64_t ray_begin, int64_t n_rays, int32_t n_samples,
                                  const float* z, int32_t z_stride, const int64_t* labels, const float* t_emb,
                                  int32_t flags, void* workspace, float* out, void* stream);
/* Gradients of sum(d_out * out) w.r.t. every parameter, written (overwritten, or added with
 * SPNERF_MLP_ACCUMULATE in `flags`) into `grad_flat` (canonical order, torch shapes,
 * contiguous) and w.r.t. t_emb (n_rays, t_dim, overwritten).  The workspace of a SAVE forward
 * serves ONE backward: the bf16 MLP's fused dX chain (option fused_bwd) writes the trunk's
 * pre-activation gradients over the saved derivatives. */
int32_t spnerf_mlp_backward(const spnerf_model_cfg* cfg, const void* packed,
                            const float* rays, int32_t ray_stride, int64_t n_rays, int32_t n_samples,
                            const int64_t* labels, const float* t_emb, int32_t flags,
                            void* workspace, const float* d_out, float* grad_flat, float* grad_t_emb,
                            void* stream);

/* The trunk layers' weight gradients (fc_net.2i.weight / .bias, without the per-ray semantic
 * columns) and those of sun_v_net.2 / .4 (present in every pass) of up to n_seg deferred
 * backwards (SPNERF_MLP_DEFER_TRUNK_WGRAD), added into grad_flat:
 * the points of two workspaces (e.g. a render's main and solar-correction passes, rendering.py:
 * 165-177, whose backwards both reach the same trunk) run as ONE weight-gradient GEMM per layer —
 * half the launches and split reductions of one GEMM per pass.  n_rays / n_samples / flags are
 * those of each workspace's forward.  n_seg = 0: returns 1 if a backward may defer under the
 * current options (the bf16 MLP with its fused dX chain), else 0. */
int32_t spnerf_mlp_trunk_wgrad(const spnerf_model_cfg* cfg, int32_t n_seg, void* const* workspaces,
                               const int64_t* n_rays, const int32_t* n_samples, const int32_t* flags,
                               float* grad_flat, void* stream);

/* ---- compositing: inference() (spnerf.py:109-157) --------------------------------------- */
/* noise (n_rays, n_samples) N(0,1) draws scaled by noise_std, or NULL with rng set: drawn on the
 * device (the backward must get the same rng) */
int32_t spnerf_composite_forward(int64_t n_rays, int32_t n_samples, const float* z, const float* out,
                                 int32_t n_out, const float* noise, float noise_std, int32_t sem_col,
                                 int32_t n_sem, int32_t flags, float* rgb, float* depth, float* weights,
                                 float* transparency, float* sem_logits, const spnerf_rng* rng, void* stream);
/* d_out (P, n_out) receives the gradient w.r.t. out (sigma, albedo, sun, sky, sem columns;
 * other columns are zeroed).  Any upstream gradient pointer may be NULL (= zero). */
int32_t spnerf_composite_backward(int64_t n_rays, int32_t n_samples, const float* z, const float* out,
                                  int32_t n_out, const float* noise, float noise_std, int32_t sem_col,
                                  int32_t n_sem, int32_t flags, const float* g_rgb, const float* g_depth,
                                  const float* g_weights, const float* g_transparency, const float* g_sem,
                                  float* d_out, const spnerf_rng* rng, void* stream);

/* ---- training losses (modules/metrics.py as main.py:125-174 combines them) ------------------
 * loss = SNerfLoss colour MSE (rgb, target (B,3); rgb NULL = off)                  metrics.py:27-45
 *      + solar_correction terms 2, 3 (lambda_sc > 0; sun_sc[(r*S+s)*ld_sun], T_sc, w_sc (B,S))  :17-24
 *      + DepthLoss subset MSE form (lambda_ds > 0; depth (B), z, w (B,S), target depth / weight at
 *        stride ld_td, valid_depth int64, target_std)                              :82-132,151-153
 *      + lambda_ss * SemanticLoss cross-entropy, ignore_index -100 (logits (B,C) NULL = off)  :162-183
 * The CE mean runs over the valid labels of labels_global[0..n_global) divided by `world` (data
 * parallelism: the ranks' losses average to the global loss; single process: labels_global =
 * labels, world = 1).  loss_out (device, 7 floats): [0] loss, [1..5] colour, sc2, sc3, depth, CE,
 * [6] the CE denominator.  Deterministic (fixed-order partial sums in `workspace`).  The
 * backward writes the gradients of g_loss[0] * loss w.r.t. rgb, sun_sc (dense (B,S)), depth and
 * logits, reading loss_out[6]. */
int64_t spnerf_render_loss_workspace_bytes(int64_t n_rays);
int32_t spnerf_render_loss_forward(int64_t n_rays, int32_t n_samples, int32_t n_classes, const float* rgb,
                                   const float* target, float lambda_sc, const float* sun_sc, int32_t ld_sun,
                                   const float* T_sc, const float* w_sc, float lambda_ds, const float* depth,
                                   const float* z, const float* w, const float* target_depth,
                                   const float* target_weight, int32_t ld_td, const int64_t* valid_depth,
                                   const float* target_std, float lambda_ss, const float* logits,
                                   const int64_t* labels, const int64_t* labels_global, int64_t n_global,
                                   int32_t world, void* workspace, float* loss_out, void* stream);
int32_t spnerf_render_loss_backward(int64_t n_rays, int32_t n_samples, int32_t n_classes, const float* rgb,
                                    const float* target, float lambda_sc, const float* sun_sc, int32_t ld_sun,
                                    const float* T_sc, const float* w_sc, float lambda_ds, const float* depth,
                                    const float* z, const float* w, const float* target_depth,
                                    const float* target_weight, int32_t ld_td, const int64_t* valid_depth,
                                    const float* target_std, float lambda_ss, const float* logits,
                                    const int64_t* labels, const float* loss_out, const float* g_loss,
                                    float* d_rgb, float* d_sun_sc, float* d_depth, float* d_logits, void* stream);

/* ---- sample generation (rendering.py) --------------------------------------------------- */
/* stratified jittered depths, perturb = 1 (rendering.py:131-144); u (n_rays, n) in [0,1), or
 * NULL with rng set (drawn on the device) */
int32_t spnerf_sample_stratified(int64_t n_rays, int32_t n_samples, const float* rays, int32_t ray_stride,
                                 const float* u, float* z, const spnerf_rng* rng, void* stream);
/* GenerateGuidedSamples + sort + merge (rendering.py:92-116,165-167): 3-sigma window around
 * the pass-1 depth, replaced by the GT window on rays with valid_depth > 0 (valid_depth may be
 * NULL = test mode), clamped to clamp_nf[0..1] (device; the chunk's first-ray near/far,
 * rendering.py:95,113).  u_pred / u_gt are (n_rays, n).  Writes z_sorted = sort([z, z2]) and
 * z_unsort = [z, sort(z2)], both (n_rays, 2n). */
int32_t spnerf_sample_guided(int64_t n_rays, int32_t n_samples, const float* z, const float* depth,
                             const float* weights, const float* clamp_nf, const int64_t* valid_depth,
                             const float* target_depths, int32_t td_stride, const float* target_std,
                             const float* u_pred, const float* u_gt, float* z_sorted, float* z_unsort,
                             const spnerf_rng* rng, void* stream);
/* sample_pdf (rendering.py:14-55): bins (n_rays, n_bins+1), weights (n_rays, n_bins),
 * u (n_rays, n_imp) → samples (n_rays, n_imp). n_bins+1 <= 256, n_imp <= 256. */
int32_t spnerf_sample_pdf(int64_t n_rays, int32_t n_bins, const float* bins, const float* weights,
                          int32_t n_imp, const float* u, float eps, float* samples, const spnerf_rng* rng,
                          void* stream);
/* sample_3sigma (rendering.py:58-73): low/high (n_rays), u (n_rays, n) → (n_rays, n) */
int32_t spnerf_sample_3sigma(int64_t n_rays, int32_t n, const float* low, const float* high,
                             const float* clamp_nf, const float* u, float* out, void* stream);
/* row-wise ascending sort of (n_rays, n) floats, n <= 256 (torch.sort(-1) values) */
int32_t spnerf_sort_rows(int64_t n_rays, int32_t n, const float* in, float* out, void* stream);
/* rendering.py:165-168: the main pass's rows in the sorted depth order, gathered from two segments
 * of MLP rows — out1 (n_rays*s1, n_out): pass 1's stratified samples, s1 per ray; out2
 * (n_rays*s2, n_out): the guided samples, s2 per ray — by the ranks of z_unsort = [z | sorted
 * z_2] (n_rays, s1+s2), the reference's z_vals_unsort.  out_sorted (n_rays*(s1+s2), n_out).  The
 * backward scatters the sorted rows' gradients d_sorted back into the segments' rows. */
int32_t spnerf_merge_samples(int64_t n_rays, int32_t s1, int32_t s2, const float* z_unsort, const float* out1,
                             const float* out2, int32_t n_out, float* out_sorted, void* stream);
int32_t spnerf_merge_samples_backward(int64_t n_rays, int32_t s1, int32_t s2, const float* z_unsort,
                                      const float* d_sorted, int32_t n_out, float* d_out1, float* d_out2, void* stream);

/* ---- RPC camera rays: get_rays + normalize_rays + get_sun_dirs (datasets/satellite_scene.py:21-68,
 *      :415-425, :449-473; modules/utils.py:59-100).  rpc = 90 host doubles: row/col/lat/lon/alt
 *      offsets, then row/col/lat/lon/alt scales, then row_num, row_den, col_num, col_den (20 each,
 *      RPC00B order); rescaled for `downscale` like utils.rescale_rpc(rpc, 1/downscale).  Pixels:
 *      the rectangle [row0, row0+n_rows) x [col0, col0+n_cols) in row-major order, or the device
 *      list `pixels` of (col, row) int32 pairs.  center (3 host floats) == NULL skips the fp32
 *      normalisation; sun = 3 host floats (needed when ray_stride >= 11). */
int32_t spnerf_rpc_rays(const double* rpc, double downscale, double min_alt, double max_alt, int32_t row0,
                        int32_t col0, int32_t n_rows, int32_t n_cols, const int32_t* pixels, int64_t n_pixels,
                        const float* center, float range, const float* sun, float* rays, int32_t ray_stride,
                        void* stream);

/* ---- DSM extraction from a rendered depth (datasets/satellite_scene.py:475-568,
 *      modules/utils.py:103-139).  spnerf_dsm_points: per ray, x = o + d·depth (normalised scene,
 *      rays of stride rs >= 6), denormalised by `range` and the 3 host doubles `center` to ECEF,
 *      then lat / lon (degrees) / alt by the reference's ecef_to_latlon_custom into lla[n][3] and
 *      UTM easting / northing / alt (WGS-84, `utm_zone`, `south`; Krüger series — pyproj is not
 *      available: parity unpinned) into ena[n][3]; either output may be NULL.
 *      spnerf_dsm_rasterize: plyflatten(cloud, xoff, yoff, resolution, xsize, ysize, radius,
 *      sigma) restated (parity unpinned): dsm[ysize][xsize] = weighted mean altitude of the
 *      points whose (2·radius+1)² window covers the cell, NaN where none; sigma = +inf for plain
 *      means; acc = 2·xsize·ysize doubles of device workspace. */
int32_t spnerf_dsm_points(const float* rays, int32_t rs, int64_t n, const float* depth, const double* center,
                          double range, int32_t utm_zone, int32_t south, double* lla, double* ena, void* stream);
int32_t spnerf_dsm_rasterize(const double* ena, int64_t n, double xoff, double yoff, double resolution,
                             int32_t xsize, int32_t ysize, int32_t radius, double sigma, double* acc, double* dsm,
                             void* stream);

/* ---- kernel selection (no reference counterpart: A/B switches for tests and benches) ----
 *      "fused_trunk" (1 = bf16 trunk layers 1..L-1 in one persistent LDS-resident launch,
 *      the default; 0 = layer by layer), "nt_f32_variant", "tn_f32_variant",
 *      "nt_bf16_variant", "tn_bf16_variant" (GEMM tilings), "heads_variant" (1 = prefetching
 *      output heads, forward and backward, the default; 0 = one point at a time), "l0_split" (bf16 MLP: 1 = fc_net.0
 *      on bf16 hi/lo planes, the default; 0 = fp32 MFMA), "trunk_l0" (with l0_split: 1 = fc_net.0
 *      inside the fused trunk launch when nothing is saved, the default; 2 = always; 0 = never).
 *      Process-wide; unknown names fail. */
int32_t spnerf_set_option(const char* name, int32_t value);
int32_t spnerf_get_option(const char* name, int32_t* value);

/* ---- optimizer step (reference main.py:97: torch.optim.Adam; no reference kernel) -------
 * One Adam step over n fp32 tensors (device pointers; exp_avg / exp_avg_sq zero-initialised by
 * the caller before step 1), torch's arithmetic with bias corrections for `step` (>= 1). */
int32_t spnerf_adam_step(int32_t n, void* const* params, const void* const* grads, void* const* exp_avg,
                         void* const* exp_avg_sq, const int64_t* numel, double lr, double beta1, double beta2,
                         double eps, int32_t step, void* stream);

/* ---- batch gather (reference main.py:108-115, satellite_scene.py:577-592: the DataLoader's
 * per-ray batch; here the dataset's fields stay resident in HBM) ----------------------------------
 * For nfields <= 8 fields f: dst[f] row i = src[f] row idx[i], i < n, rows of row_bytes[f] bytes
 * (a positive multiple of 4; 4-byte aligned tensors).  An index outside [0, src_rows[f]) leaves
 * its destination row untouched (torch indexing would raise; the caller's sampler draws in range).
 * One launch for all fields. */
int32_t spnerf_gather_rows(const int64_t* idx, int64_t n, int32_t nfields, const void* const* src,
                           const int64_t* src_rows, const int32_t* row_bytes, void* const* dst, void* stream);

/* ---- a render's random-state step (the on-device Philox state of spnerf_rng above): state[1] += 1,
 * then snap[0..1] = state[0..1], in one launch on `stream` — the render's kernels (and its
 * backward's) read the snapshot, so a later render advancing the state changes none of its draws.
 * Replaces the torch in-place add and clone of the host binding (rng.py PhiloxRandom.begin_render):
 * one launch instead of two per training step.  state and snap: device int64[2]. */
int32_t spnerf_rng_begin(int64_t* state, int64_t* snap, void* stream);

/* ---- gradient readiness marks for data parallelism (no reference counterpart: the reference
 *      trains on one GPU, main.py:322-337).  A backward passes n_marks = layers + 2 points after
 *      which groups of parameter gradients are final: mark 0 after the output heads', mark
 *      1 + (layers-1-i) after trunk layer i's, mark layers+1 at its end (per-ray parameters).
 *      spnerf_grad_marks fills mark_of_param[idx] (canonical order) with the mark after which
 *      parameter idx receives no more writes from a main or a solar-pass backward and returns
 *      n_marks.  While armed, every spnerf_mlp_backward (and spnerf_mlp_trunk_wgrad) records the
 *      library's mark events (one set per device) on its stream, and spnerf_grad_mark_wait makes
 *      `stream` wait for the latest record of `mark`: an all-reduce issued behind it overlaps the
 *      rest of the backward.  Under HIP-graph capture a mark is a dependency edge of the graph
 *      being captured, so the waiting stream's work must be captured into the same graph. */
int32_t spnerf_grad_marks(const spnerf_model_cfg* cfg, int32_t* mark_of_param, int32_t n_params);
int32_t spnerf_grad_marks_arm(int32_t on);
int32_t spnerf_grad_mark_wait(int32_t mark, void* stream);
/* Device `device`'s mark `mark`: 1 when its latest record has completed, 0 while it is pending,
 * 2 when it was never recorded (or the device's mark events do not exist yet: a query never
 * creates them).  Safe from any host thread — the device is named, not taken from the calling
 * thread — so a hung step's diagnosis (bench.py's step watchdog thread) reports the marks an eager
 * backward on that rank's GPU reached.  Replays of a captured graph do not record them. */
int32_t spnerf_grad_mark_query(int32_t device, int32_t mark);

/* ---- in-library kernel timing (HIP events on the launch stream) ------------------------- */
int32_t spnerf_prof_enable(int32_t on);
int32_t spnerf_prof_reset(void);
/* Totals over the recorded launches of one kernel class ("gemm_nt_f32", "gemm_tn_bf16d",
 * "composite_fwd", ...: one class per kernel function, the DMA NT GEMM's x Dmul instance as
 * "gemm_nt_bf16d_dmul").  Synchronises the recorded events. */
int32_t spnerf_prof_read(const char* kernel_class, int64_t* launches, double* total_ms, double* total_flop,
                         double* total_bytes);
/* The names of the classes recorded since the last reset, comma-separated, into buf (cap bytes). */
int32_t spnerf_prof_classes(char* buf, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* SPNERF_AMD_H */
