// Parameter / packed-weight / workspace layouts (host only).
#include "mlp_layout.h"

#include <algorithm>

#include "gemm_bf16.h"
#include "gemm_f32.h"
#include "trunk.h"

namespace spn {

static inline int pad32(int x) { return (x + 31) / 32 * 32; }

int32_t make_dims(const spnerf_model_cfg* c, Dims* d) {
    SPN_ARG(c != nullptr, "cfg is NULL");
    SPN_ARG(c->width >= 32 && c->width % 64 == 0, "width %d must be a multiple of 64", c->width);
    SPN_ARG(c->layers >= 2 && c->layers <= 16, "layers %d out of range", c->layers);
    SPN_ARG(c->skip < c->layers && c->skip != 0, "skip %d must be in [1, layers) or -1", c->skip);
    SPN_ARG(c->n_freq >= 0 && c->n_freq <= 16, "n_freq %d out of range", c->n_freq);
    SPN_ARG(c->sem_classes >= 0 && c->sem_classes <= 32, "sem_classes %d out of range", c->sem_classes);
    SPN_ARG((c->sem_classes == 0) == (c->sem_dim == 0), "sem_classes/sem_dim mismatch");
    SPN_ARG(c->sem_dim <= 64, "sem_dim %d too large", c->sem_dim);
    SPN_ARG(!c->beta || (c->t_dim > 0 && c->t_dim <= 64), "t_dim %d out of range", c->t_dim);
    SPN_ARG(c->dtype == 0 || c->dtype == 1, "dtype %d not supported (0 = fp32, 1 = bf16)", c->dtype);
    d->W = c->width;
    d->H = c->width / 2;
    d->L = c->layers;
    d->skip = c->skip;
    d->K0 = c->n_freq > 0 ? 6 * c->n_freq : 3;
    d->K0p = pad32(d->K0);
    d->sem = c->sem_classes > 0;
    d->C = c->sem_classes;
    d->sd = c->sem_dim;
    d->beta = c->beta != 0;
    d->td = d->beta ? c->t_dim : 0;
    d->NG = d->W + (d->sem ? d->H : 0);
    d->NQ = 2 * d->H + (d->beta ? d->H : 0);
    d->NO = 8 + (d->beta ? 1 : 0) + d->C;
    d->sem_col = 8 + (d->beta ? 1 : 0);
    d->HP = 6 + d->C;
    d->bf = c->dtype == 1;
    return SPNERF_OK;
}

std::vector<PSpec> param_specs(const Dims& d, PIdx* ix) {
    std::vector<PSpec> v;
    PIdx tmp;
    PIdx& x = ix ? *ix : tmp;
    auto add = [&](const std::string& n, int64_t r, int64_t c) {
        v.push_back(PSpec{n, r, c, 0});
        return (int)v.size() - 1;
    };
    const int W = d.W, H = d.H, in = d.K0 + d.sd;
    if (d.sem) x.emb = add("semantic_embedding.weight", d.C + 1, d.sd);
    x.fcW.clear();
    x.fcb.clear();
    for (int i = 0; i < d.L; ++i) {
        const int fan = i == 0 ? in : (i == d.skip ? W + in : W);
        x.fcW.push_back(add("fc_net." + std::to_string(2 * i) + ".weight", W, fan));
        x.fcb.push_back(add("fc_net." + std::to_string(2 * i) + ".bias", W, 0));
    }
    x.sigW = add("sigma_from_xyz.0.weight", 1, W);
    x.sigb = add("sigma_from_xyz.0.bias", 1, 0);
    x.featW = add("feats_from_xyz.weight", W, W);
    x.featb = add("feats_from_xyz.bias", W, 0);
    if (d.sem) {
        x.m1W = add("logit_from_label.0.weight", H, W);
        x.m1b = add("logit_from_label.0.bias", H, 0);
        x.m2W = add("logit_from_label.2.weight", d.C, H);
        x.m2b = add("logit_from_label.2.bias", d.C, 0);
    }
    x.r1W = add("rgb_from_xyzdir.0.weight", H, W);
    x.r1b = add("rgb_from_xyzdir.0.bias", H, 0);
    x.r2W = add("rgb_from_xyzdir.2.weight", 3, H);
    x.r2b = add("rgb_from_xyzdir.2.bias", 3, 0);
    x.s1W = add("sun_v_net.0.weight", H, W + 3);
    x.s1b = add("sun_v_net.0.bias", H, 0);
    x.s2W = add("sun_v_net.2.weight", H, H);
    x.s2b = add("sun_v_net.2.bias", H, 0);
    x.s3W = add("sun_v_net.4.weight", H, H);
    x.s3b = add("sun_v_net.4.bias", H, 0);
    x.s4W = add("sun_v_net.6.weight", 1, H);
    x.s4b = add("sun_v_net.6.bias", 1, 0);
    x.k1W = add("sky_color.0.weight", H, 3);
    x.k1b = add("sky_color.0.bias", H, 0);
    x.k2W = add("sky_color.2.weight", 3, H);
    x.k2b = add("sky_color.2.bias", 3, 0);
    if (d.beta) {
        x.b1W = add("beta_from_xyz.0.weight", H, d.td + W);
        x.b1b = add("beta_from_xyz.0.bias", H, 0);
        x.b2W = add("beta_from_xyz.2.weight", 1, H);
        x.b2b = add("beta_from_xyz.2.bias", 1, 0);
    }
    int64_t off = 0;
    for (auto& p : v) {
        p.off = off;
        off += p.numel();
    }
    return v;
}

Packed packed_layout(const Dims& d) {
    Packed k;
    int64_t off = 0;
    auto take = [&](int64_t n) {
        const int64_t o = off;
        off += (n + 63) / 64 * 64;  // keep every block 256-B aligned
        return o;
    };
    const int W = d.W, H = d.H;
    for (int i = 0; i < d.L; ++i) {
        const int Kp = i == 0 ? d.K0p : (i == d.skip ? W + d.K0p : W);
        k.Kp.push_back(Kp);
        k.Wt.push_back(take((int64_t)W * Kp));
        k.bt.push_back(take(W));
        k.WTt.push_back(i == 0 ? -1 : take((int64_t)W * W));
    }
    k.WG = take((int64_t)d.NG * W);
    k.bG = take(d.NG);
    k.WGT = take((int64_t)W * d.NG);
    k.WQ = take((int64_t)d.NQ * W);
    k.bQ = take(d.NQ);
    k.WQT = take((int64_t)W * d.NQ);
    k.Ws2 = take((int64_t)H * H);
    k.bs2 = take(H);
    k.Ws2T = take((int64_t)H * H);
    k.Ws3 = take((int64_t)H * H);
    k.bs3 = take(H);
    k.Ws3T = take((int64_t)H * H);
    k.wsig = take(W);
    k.bsig = take(1);
    k.Wr2 = take(3 * H);
    k.br2 = take(3);
    k.ws4 = take(H);
    k.bs4 = take(1);
    k.Wm2 = take((int64_t)(d.C ? d.C : 1) * H);
    k.bm2 = take(d.C ? d.C : 1);
    k.wb2 = take(H);
    k.bb2 = take(1);
    k.Wk1 = take(3 * H);
    k.bk1 = take(H);
    k.Wk2 = take(3 * H);
    k.bk2 = take(3);
    k.Wsem0 = take((int64_t)W * (d.sd ? d.sd : 1));
    k.Wsem4 = take((int64_t)W * (d.sd ? d.sd : 1));
    k.emb = take((int64_t)(d.C + 1) * (d.sd ? d.sd : 1));
    k.Wsun = take(3 * H);
    k.Wtt = take((int64_t)H * (d.td ? d.td : 1));
    if (d.bf) {
        auto take16 = [&](int64_t n) { return 2 * take((n + 1) / 2); };
        const bool fused = trunk_bf16_supported(W, d.L, d.skip, d.K0p);
        for (int i = 0; i < d.L; ++i) {
            k.Wt16.push_back(i == 0 ? -1 : take16((int64_t)W * k.Kp[i]));
            k.WTt16.push_back(i == 0 ? -1 : take16((int64_t)W * W));
            k.Wf16.push_back(!fused ? -1 : take16((int64_t)W * (i == 0 ? 4 * k.Kp[0] : k.Kp[i])));
            k.Wb16.push_back(!fused || i == 0 ? -1 : take16((int64_t)W * W));
        }
        k.WG16 = take16((int64_t)d.NG * W);
        k.WGT16 = take16((int64_t)W * d.NG);
        k.WQ16 = take16((int64_t)d.NQ * W);
        k.WQT16 = take16((int64_t)W * d.NQ);
        k.Ws2_16 = take16((int64_t)H * H);
        k.Ws2T16 = take16((int64_t)H * H);
        k.Ws3_16 = take16((int64_t)H * H);
        k.Ws3T16 = take16((int64_t)H * H);
        k.W0s16 = take16((int64_t)W * 4 * k.Kp[0]);
        if (heads_bf16_shape_ok(d)) {
            if (d.sem) k.Fsem16 = take16((int64_t)H * W);
            k.Ffeat16 = take16((int64_t)W * W);
            k.FQ16 = take16((int64_t)2 * H * W);
            k.Fs2_16 = take16((int64_t)H * H);
            k.Fs3_16 = take16((int64_t)H * H);
            k.FQs16 = take16((int64_t)H * W);
            k.Fnar16 = take16((int64_t)32 * (W + 2 * H));
            if (!d.beta && kAblBuild) {  // the training heads' fused dX chain (an ablation-build kernel)
                k.Bs3_16 = take16((int64_t)H * H);
                k.Bs2_16 = take16((int64_t)H * H);
                k.BQ16 = take16((int64_t)W * d.NQ);
                k.BG16 = take16((int64_t)W * d.NG);
            }
        }
    }
    k.total = off;
    return k;
}

WS ws_layout(const Dims& d, int64_t n_rays, int32_t S, int32_t flags) {
    WS w{};
    const int64_t P = n_rays * S, B = n_rays;
    const bool save = flags & SPNERF_MLP_SAVE;
    w.P = P;
    w.B = B;
    int64_t off = 0;
    auto take = [&](int64_t n) {
        const int64_t o = off;
        off += (n + 63) / 64 * 64;
        return o;
    };
    // activation-sized buffers: fp32, or bf16 (half the floats) in the bf16 MLP
    auto act = [&](int64_t n) { return d.bf ? take((n + 1) / 2) : take(n); };
    const int W = d.W, H = d.H;
    w.X0 = take(P * d.K0p);
    w.X0b = d.bf ? act(P * d.K0p) : -1;
    w.X0s = d.bf ? act(P * 4 * d.K0p) : -1;
    if (save) {
        for (int i = 0; i < d.L; ++i) w.Hb.push_back(act(P * W));
        for (int i = 0; i < d.L; ++i) w.Db.push_back(act(P * W));
    } else {
        for (int i = 0; i < 3; ++i) w.Hb.push_back(act(P * W));
    }
    w.G = act(P * d.NG);
    w.DG = save ? act(P * d.NG) : -1;
    w.Q = act(P * d.NQ);
    w.DQ = save ? act(P * d.NQ) : -1;
    if (save) {
        w.S2 = act(P * H);
        w.DS2 = act(P * H);
        w.S3 = act(P * H);
        w.DS3 = act(P * H);
    } else {
        w.S2 = w.S3 = w.DS2 = w.DS3 = -1;  // ping-pong buffers are used
    }
    w.hsave = take(P * 8);
    w.rb0 = take(B * W);
    w.rb4 = take(B * W);
    w.rbQ = take(B * d.NQ);
    w.skyh = take(B * H);
    w.sky = take(B * 4);
    if (save) {
        w.dZG = act(P * d.NG);
        w.dZQ = act(P * d.NQ);
        w.dS3 = act(P * H);
        w.dS2 = act(P * H);
        w.dZa = act(P * W);   // trunk dZ: three buffers in rotation, so the weight gradient of
        w.dZb = act(P * W);   // layer i (side stream) reads dZ_i while the main stream writes
        w.dZc = act(P * W);   // dZ_{i-1} into another
        w.hpre = take(P * d.HP);
        // largest TN slab over every weight-gradient GEMM of the backward
        int64_t slab = 0, slab_b = 0;
        auto need = [&](int N, int K) {
            // bf16: either TN tiling may run (tn_bf16_variant can change after the layout is made)
            const int sp = d.bf ? std::max(tn_splits_bf16((int)P, N, K, 1, -1, kLayoutCus),
                                           tn_splits_bf16((int)P, N, K, 2, 1, kLayoutCus))
                                : tn_splits((int)P, N, K);
            slab = std::max(slab, (int64_t)sp * N * K);
            slab_b = std::max(slab_b, (int64_t)sp * N);
        };
        for (int i = 0; i < d.L; ++i) need(W, i == 0 ? d.K0p : (i == d.skip ? W + d.K0p : W));
        need(d.NG, W);
        need(d.NQ, W);
        need(H, H);
        if (d.bf && d.W % 256 == 0) {
            // grouped weight gradients (mlp.hip trunk_wgrad, option tn_group): up to
            // kTnGroupRounds x kLayoutCus 256 x 256 blocks of the DMA kernel, each its own slab tile,
            // over both passes' points (at most 2P here; trunk_wgrad clamps to this capacity)
            const int64_t blocks = std::min<int64_t>((int64_t)kTnGroupRounds * kLayoutCus,
                                                     (int64_t)kTnGroup * 4 * ((2 * P + 1023) / 1024));
            slab = std::max(slab, blocks * 256 * 256);
            slab_b = std::max(slab_b, blocks * 256);
        }
        w.slab_n = slab;
        w.slab_b_n = slab_b;
        w.slab = take(slab);
        w.slab_b = take(slab_b);
        w.RQ = take(B * d.NQ);
        w.R0 = take(B * W);
        w.R4 = take(B * W);
        // per-64-point-tile column sums of dZ_0 / dZ_skip (tile_colsum order), summed per ray
        w.Rp0 = take((P + 63) / 64 * W);
        w.Rp4 = take((P + 63) / 64 * W);
        w.skyd = take(B * 4);
        w.skydh = take(B * H);
        w.gemb = take(B * (d.sd ? d.sd : 1));
        w.embr = take(B * (d.sd ? d.sd : 1));
        // skinny slabs: one point reduction at a time, or the per-ray batch (≤ kSkinnyMulti tasks of
        // ≤ 9 rows x max(W, H) columns each, mlp.hip SkinnyBatch)
        // chunks of any row count up to P (resp. B): skinny_chunk's bound
        const int64_t cP = std::min<int64_t>((P + 63) / 64, 768), cB = std::min<int64_t>((B + 63) / 64, 768);
        w.sk_slab_n = std::max(cP * 9 * W, cB * kSkinnyMulti * 9 * W);
        w.sk_slab_b_n = std::max(cP * 9, cB * kSkinnyMulti * 9);
        w.sk_slab = take(w.sk_slab_n);
        w.sk_slab_b = take(w.sk_slab_b_n);
    }
    w.total = off;
    return w;
}

WS ws_window(const Dims& d, const WS& full, int64_t r0, int64_t n, int32_t S) {
    WS w = full;
    const int64_t p0 = r0 * S;
    w.P = n * S;
    w.B = n;
    // point-major rows: fp32, or bf16 at half the floats (every width here is even)
    auto pts = [&](int64_t& off, int64_t width, bool act) {
        if (off >= 0) off += act && d.bf ? p0 * width / 2 : p0 * width;
    };
    auto rows = [&](int64_t& off, int64_t width) {
        if (off >= 0) off += r0 * width;
    };
    pts(w.X0, d.K0p, false);
    pts(w.X0b, d.K0p, true);
    pts(w.X0s, 4 * d.K0p, true);
    for (auto& o : w.Hb) pts(o, d.W, true);
    for (auto& o : w.Db) pts(o, d.W, true);
    pts(w.G, d.NG, true);
    pts(w.DG, d.NG, true);
    pts(w.Q, d.NQ, true);
    pts(w.DQ, d.NQ, true);
    pts(w.S2, d.H, true);
    pts(w.DS2, d.H, true);
    pts(w.S3, d.H, true);
    pts(w.DS3, d.H, true);
    pts(w.hsave, 8, false);
    rows(w.rb0, d.W);
    rows(w.rb4, d.W);
    rows(w.rbQ, d.NQ);
    rows(w.skyh, d.H);
    rows(w.sky, 4);
    return w;
}

}  // namespace spn
