// mastering.hip — host side of the C-ABI (include/mastering.h): device buffers,
// the launch sequence of the chain, loudness gating, event timing and RCCL.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/mastering.h"
#include "kernels.hip"
#include "compressor.hip"
#include "scan.hip"

using namespace mm;

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
};

struct PendingEvent {
    std::string name;
    hipEvent_t a, b;
};

struct KStat {
    double ms = 0.0;
    int64_t n = 0;
};

}  // namespace

struct mm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    char err[512] = {0};
    std::map<std::string, DevBuf> bufs;
    // staged job geometry (mm_stage_chunks -> mm_hop_energies / mm_finalize)
    bool staged = false;
    mm_job job{};
    int64_t G = 0;
    short2 *mix = nullptr;
    // timing
    bool timing = false;
    std::vector<PendingEvent> pending;
    std::vector<hipEvent_t> free_events;
    std::map<std::string, KStat> stats;
    std::vector<std::string> stat_order;
    // host tables already resident on the device
    const double *lut_src[3] = {nullptr, nullptr, nullptr};
    std::map<std::string, std::vector<double>> mats_cache;
    // rccl
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
};

static int set_err(mm_ctx *c, int code, const char *fmt, ...) {
    if (c) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(c->err, sizeof(c->err), fmt, ap);
        va_end(ap);
    }
    return code;
}

#define HIPCHK(ctx, expr)                                                                    \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err(ctx, MM_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                           __FILE__, __LINE__);                                              \
    } while (0)

template <typename T>
static int get_buf(mm_ctx *c, const char *name, size_t count, T **out) {
    DevBuf &b = c->bufs[name];
    size_t bytes = std::max<size_t>(count * sizeof(T), 256);
    if (b.cap < bytes) {
        if (b.p) HIPCHK(c, hipFree(b.p));
        b.p = nullptr;
        b.cap = 0;
        HIPCHK(c, hipMalloc(&b.p, bytes));
        b.cap = bytes;
    }
    *out = reinterpret_cast<T *>(b.p);
    return MM_OK;
}

static hipEvent_t take_event(mm_ctx *c) {
    if (!c->free_events.empty()) {
        hipEvent_t e = c->free_events.back();
        c->free_events.pop_back();
        return e;
    }
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Launch helper: records HIP events around the kernel on the context stream
// when timing is enabled.
template <typename Kern, typename... Args>
static int launch(mm_ctx *c, const char *name, Kern k, dim3 grid, dim3 block, size_t lds, Args... args) {
    hipEvent_t a = nullptr, b = nullptr;
    if (c->timing) {
        a = take_event(c);
        b = take_event(c);
        if (a) hipEventRecord(a, c->stream);
    }
    hipLaunchKernelGGL(k, grid, block, lds, c->stream, args...);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(c, MM_ERR_HIP, "launch %s: %s", name, hipGetErrorString(e));
    if (c->timing && a && b) {
        hipEventRecord(b, c->stream);
        c->pending.push_back({name, a, b});
    }
    return MM_OK;
}

static void resolve_events(mm_ctx *c) {
    for (auto &p : c->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            auto it = c->stats.find(p.name);
            if (it == c->stats.end()) {
                c->stat_order.push_back(p.name);
                it = c->stats.emplace(p.name, KStat{}).first;
            }
            it->second.ms += ms;
            it->second.n += 1;
        }
        c->free_events.push_back(p.a);
        c->free_events.push_back(p.b);
    }
    c->pending.clear();
}

#define RET(expr)                  \
    do {                           \
        int r_ = (expr);           \
        if (r_ != MM_OK) return r_; \
    } while (0)

static inline unsigned blocks_for(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

// ------------------------------------------------------------------ scan
// Carry-in state of every tile (scan.hip): block-local scan, block-carry scan,
// apply.  The transition powers are uploaded only when they change.
static int run_scan(mm_ctx *c, const char *name, const mm_iir &f, int dim, int ch, int64_t line_tiles,
                    int64_t G, const double *z, double *s, const double *init, double *line_end) {
    const int64_t nblk = (G + SCAN_BLOCK - 1) / SCAN_BLOCK;
    const int64_t c_needed = std::max<int64_t>(1, (nblk + SCAN_THREADS - 1) / SCAN_THREADS);
    if (f.scan_c != c_needed)
        return set_err(c, MM_ERR_ARG, "%s: block powers built for c=%d, need %lld", name, f.scan_c,
                       (long long)c_needed);
    std::vector<double> host((size_t)MAT_COUNT * 64);
    memcpy(&host[MAT_PHI * 64], f.phi, 64 * sizeof(double));
    memcpy(&host[MAT_POW2 * 64], f.phi_pow, 12 * 64 * sizeof(double));
    memcpy(&host[MAT_BLK * 64], f.phi_blk, 64 * sizeof(double));
    memcpy(&host[MAT_BLKPOW * 64], f.phi_blk_pow, 12 * 64 * sizeof(double));
    memcpy(&host[MAT_LAST * 64], f.phi_last, 64 * sizeof(double));
    const std::string key = std::string("mats_") + name;
    double *mats;
    RET(get_buf(c, key.c_str(), host.size(), &mats));
    std::vector<double> &cached = c->mats_cache[key];
    if (cached != host) {
        HIPCHK(c, hipMemcpyAsync(mats, host.data(), host.size() * sizeof(double), hipMemcpyHostToDevice,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));  // host vector is transient
        cached = host;
    }
    ScanArgs a{};
    a.dim = dim;
    a.ch = ch;
    a.line_tiles = line_tiles;
    a.G = G;
    a.nblk = nblk;
    a.c = c_needed;
    a.mats = mats;
    a.z = z;
    a.s = s;
    a.init = init;
    a.line_end = line_end;
    RET(get_buf(c, (key + "_need").c_str(), (size_t)G * ch, &a.need));
    RET(get_buf(c, (key + "_agg").c_str(), (size_t)nblk * ch * dim, &a.agg));
    RET(get_buf(c, (key + "_aggf").c_str(), (size_t)nblk * ch, &a.agg_f));
    RET(get_buf(c, (key + "_carry").c_str(), (size_t)nblk * ch * dim, &a.carry));
    const dim3 gl((unsigned)nblk, (unsigned)ch);
    if (dim == 8) {
        RET(launch(c, name, scan_local_kernel<8>, gl, dim3(SCAN_BLOCK), 0, a));
        RET(launch(c, name, scan_blocks_kernel<8>, dim3((unsigned)ch), dim3(SCAN_THREADS), 0, a));
        return launch(c, name, scan_apply_kernel<8>, gl, dim3(SCAN_BLOCK), 0, a);
    }
    if (dim == 4) {
        RET(launch(c, name, scan_local_kernel<4>, gl, dim3(SCAN_BLOCK), 0, a));
        RET(launch(c, name, scan_blocks_kernel<4>, dim3((unsigned)ch), dim3(SCAN_THREADS), 0, a));
        return launch(c, name, scan_apply_kernel<4>, gl, dim3(SCAN_BLOCK), 0, a);
    }
    return set_err(c, MM_ERR_ARG, "scan dim %d", dim);
}

static int validate(mm_ctx *c, const mm_job *j) {
    if (!j) return set_err(c, MM_ERR_ARG, "null job");
    if (j->channels != 1 && j->channels != 2) return set_err(c, MM_ERR_ARG, "channels must be 1 or 2");
    if (j->tile < 16 || j->tile > 4096) return set_err(c, MM_ERR_ARG, "tile %d out of range", j->tile);
    if (j->tiles_per_chunk < 1) return set_err(c, MM_ERR_ARG, "tiles_per_chunk < 1");
    if (j->frames_proc < 0 || j->frames_in < 0) return set_err(c, MM_ERR_ARG, "negative frame count");
    if (j->eq.nsec < 0 || j->eq.nsec > 4) return set_err(c, MM_ERR_ARG, "eq.nsec %d", j->eq.nsec);
    if (j->multiband_on) {
        if (j->xover.nsec != 4 || j->xover.nsec_branch0 != 2) return set_err(c, MM_ERR_ARG, "crossover must be 2+2 sections");
        for (int b = 0; b < 3; ++b) {
            if (!j->band[b].max_att) return set_err(c, MM_ERR_ARG, "band %d: missing max_att table", b);
            if (j->band[b].look < 0) return set_err(c, MM_ERR_ARG, "band %d: look < 0", b);
        }
    }
    if (j->lufs_on) {
        if (j->kweight.nsec != 2) return set_err(c, MM_ERR_ARG, "K-weighting must be 2 sections");
        if (j->n_segs < 1 || !j->seg_bounds || !j->block_lo || !j->block_hi || j->n_blocks < 1)
            return set_err(c, MM_ERR_ARG, "missing loudness geometry");
        for (int64_t s = 0; s < j->n_segs; ++s) {
            int64_t b0 = j->seg_bounds[s], b1 = std::min<int64_t>(j->seg_bounds[s + 1], j->frames_proc);
            if (b1 > b0 && b1 - b0 < j->tile && s + 1 < j->n_segs)
                return set_err(c, MM_ERR_ARG, "loudness segment %lld shorter than a tile", (long long)s);
        }
    }
    return MM_OK;
}

static void fill_sos(double dst[4][5], const mm_iir &f, int n) {
    for (int s = 0; s < 4; ++s)
        for (int k = 0; k < 5; ++k) dst[s][k] = s < n ? f.sos[s][k] : 0.0;
}

template <int NS, bool P2>
static int launch_eq_ch(mm_ctx *c, int ch, unsigned nb, const StageArgs &sa) {
    const char *nm = P2 ? "eq_pass2" : "eq_pass1";
    if (ch == 2) return launch(c, nm, eq_kernel<NS, P2, 2>, dim3(nb), dim3(256), 0, sa);
    return launch(c, nm, eq_kernel<NS, P2, 1>, dim3(nb), dim3(256), 0, sa);
}

template <bool P2>
static int launch_eq_p(mm_ctx *c, int nsec, int ch, unsigned nb, const StageArgs &sa) {
    switch (nsec) {
        case 1: return launch_eq_ch<1, P2>(c, ch, nb, sa);
        case 2: return launch_eq_ch<2, P2>(c, ch, nb, sa);
        case 3: return launch_eq_ch<3, P2>(c, ch, nb, sa);
        default: return launch_eq_ch<4, P2>(c, ch, nb, sa);
    }
}

static int launch_eq(mm_ctx *c, int nsec, bool pass2, int ch, unsigned nb, const StageArgs &sa) {
    return pass2 ? launch_eq_p<true>(c, nsec, ch, nb, sa) : launch_eq_p<false>(c, nsec, ch, nb, sa);
}

// ------------------------------------------------------------ chain A..C
static int stage_chunks(mm_ctx *c, const mm_job *j, const float *d_in) {
    RET(validate(c, j));
    const int T = j->tile, ch = j->channels, K = j->tiles_per_chunk;
    const int64_t N = j->frames_proc;
    const int64_t G = (N + T - 1) / T;
    const int64_t TG = (int64_t)T * std::max<int64_t>(G, 1);
    c->G = G;
    c->job = *j;
    c->staged = false;
    short2 *q1;
    RET(get_buf(c, "q1", TG, &q1));
    double *z8, *s8;
    RET(get_buf(c, "z8", (size_t)std::max<int64_t>(G, 1) * ch * 8, &z8));
    RET(get_buf(c, "s8", (size_t)std::max<int64_t>(G, 1) * ch * 8, &s8));
    const unsigned nb = blocks_for(std::max<int64_t>(G, 1), 256);

    StageArgs sa{};
    sa.in = d_in;
    sa.N_in = j->frames_in;
    sa.N_proc = N;
    sa.G = G;
    sa.T = T;
    sa.ch = ch;
    sa.sat.keep = j->sat_keep;
    sa.sat.mix = j->sat_mix;
    sa.sat.drive = j->sat_drive;
    sa.sat.on = j->sat_on;
    sa.width = j->width;
    sa.width_on = j->width_on && ch == 2;
    sa.z_out = z8;
    sa.s_in = s8;
    sa.q_out = q1;
    if (G > 0) {
        // --- stage A: saturation -> EQ -> width -> int16 (AME:55-63)
        if (j->eq.nsec == 0) {
            if (ch == 2) RET(launch(c, "pre_pointwise", pre_pointwise_kernel<2>, dim3(nb), dim3(256), 0, sa));
            else RET(launch(c, "pre_pointwise", pre_pointwise_kernel<1>, dim3(nb), dim3(256), 0, sa));
        } else {
            fill_sos(sa.sos, j->eq, j->eq.nsec);
            RET(launch_eq(c, j->eq.nsec, false, ch, nb, sa));
            RET(run_scan(c, "eq_scan", j->eq, 8, ch, K, G, z8, s8, nullptr, nullptr));
            RET(launch_eq(c, j->eq.nsec, true, ch, nb, sa));
        }
    }
    short2 *mix = q1;
    if (j->multiband_on && G > 0) {
        // --- stage B: crossover + band quantisation (AME:196-206)
        short2 *bands[3];
        RET(get_buf(c, "band0", TG, &bands[0]));
        RET(get_buf(c, "band1", TG, &bands[1]));
        RET(get_buf(c, "band2", TG, &bands[2]));
        StageArgs xa = sa;
        fill_sos(xa.sos, j->xover, 4);
        xa.q_in = q1;
        for (int b = 0; b < 3; ++b) xa.band_out[b] = bands[b];
        RET(launch(c, "xover_pass1", xover_kernel<false>, dim3(nb), dim3(256), 0, xa));
        RET(run_scan(c, "xover_scan", j->xover, 8, ch, K, G, z8, s8, nullptr, nullptr));
        RET(launch(c, "xover_pass2", xover_kernel<true>, dim3(nb), dim3(256), 0, xa));

        // --- stage C: 3-band compressor + overlay (AME:207-210)
        CompArgs ca{};
        ca.N_proc = N;
        ca.G = G;
        ca.T = T;
        ca.K = K;
        ca.ch = ch;
        ca.warmup = j->comp_warmup;
        ca.U = std::max(16, j->comp_super);
        const int64_t nchunks = (G + K - 1) / K;
        ca.SPC = ((int64_t)K * T + ca.U - 1) / ca.U;
        ca.GS = nchunks * ca.SPC;
        const int64_t GS = ca.GS;
        short2 *q2;
        RET(get_buf(c, "q2", TG, &q2));
        ca.q_out = q2;
        double *st, *eA, *eB, *luts, *tst;
        RET(get_buf(c, "comp_start", (size_t)3 * GS, &st));
        RET(get_buf(c, "comp_endA", (size_t)3 * GS, &eA));
        RET(get_buf(c, "comp_endB", (size_t)3 * GS, &eB));
        RET(get_buf(c, "comp_tstart", (size_t)3 * G, &tst));
        RET(get_buf(c, "comp_lut", (size_t)3 * 32769, &luts));
        unsigned int *changed;
        RET(get_buf(c, "comp_changed", 64, &changed));
        int32_t *cnt, *off, *tot;
        RET(get_buf(c, "comp_cnt", (size_t)3 * G, &cnt));
        RET(get_buf(c, "comp_off", (size_t)3 * G, &off));
        RET(get_buf(c, "comp_total", (size_t)3 * nchunks, &tot));
        for (int b = 0; b < 3; ++b) {
            uint16_t *rb;
            double *mcb;
            char nm[16];
            snprintf(nm, sizeof nm, "comp_r%d", b);
            RET(get_buf(c, nm, TG, &rb));
            snprintf(nm, sizeof nm, "comp_Mc%d", b);
            RET(get_buf(c, nm, (size_t)GS * (ca.U + 1), &mcb));  // + one padding row
            ca.r16[b] = rb;
            ca.Mc[b] = mcb;
            ca.band[b] = bands[b];
            ca.max_att[b] = luts + (size_t)b * 32769;
            // tables are immutable host arrays owned by the caller's job: upload once
            if (c->lut_src[b] != j->band[b].max_att) {
                HIPCHK(c, hipMemcpyAsync(luts + (size_t)b * 32769, j->band[b].max_att, 32769 * sizeof(double),
                                         hipMemcpyHostToDevice, c->stream));
                c->lut_src[b] = j->band[b].max_att;
            }
            ca.r0[b] = (uint32_t)j->band[b].r0;
            ca.look[b] = j->band[b].look;
            ca.attack_frames[b] = j->band[b].attack_frames;
            ca.release_frames[b] = j->band[b].release_frames;
            ca.rcp_attack[b] = 1.0 / j->band[b].attack_frames;
            ca.rcp_release[b] = 1.0 / j->band[b].release_frames;
            ca.cnt[b] = cnt + (size_t)b * G;
            ca.off[b] = off + (size_t)b * G;
            ca.total[b] = tot + (size_t)b * nchunks;
            ca.start[b] = st + (size_t)b * GS;
            ca.tstart[b] = tst + (size_t)b * G;
            ca.end_out[b] = eA + (size_t)b * GS;
        }
        const unsigned nbs = blocks_for(GS, 256);
        RET(launch(c, "comp_rms", comp_rms_kernel, dim3(nb, 3), dim3(256), 0, ca));
        RET(launch(c, "comp_offsets", comp_offsets_kernel, dim3((unsigned)nchunks, 3), dim3(1024), 0, ca));
        RET(launch(c, "comp_compact", comp_compact_kernel, dim3(nb, 3), dim3(256), 0, ca));
        RET(launch(c, "comp_pass0", comp_pass0_kernel, dim3(nbs, 3), dim3(256), 0, ca));
        // Jacobi sweeps queued in batches: sweep k writes flag k, and exits at once
        // if sweep k-1 changed nothing; one host sync per batch.
        const int batch = 16;
        int iters = 0;
        double *cur = eA, *nxt = eB;
        bool done = false;
        while (!done) {
            HIPCHK(c, hipMemsetAsync(changed, 0, batch * sizeof(unsigned int), c->stream));
            for (int k = 0; k < batch; ++k) {
                for (int b = 0; b < 3; ++b) {
                    ca.end_in[b] = cur + (size_t)b * GS;
                    ca.end_out[b] = nxt + (size_t)b * GS;
                }
                ca.changed = changed + k;
                const unsigned int *prevf = k > 0 ? changed + (k - 1) : nullptr;
                RET(launch(c, "comp_fix", comp_fix_kernel, dim3(nbs, 3), dim3(256), 0, ca, prevf));
                std::swap(cur, nxt);
            }
            unsigned int h[batch];
            HIPCHK(c, hipMemcpyAsync(h, changed, sizeof h, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            for (int k = 0; k < batch; ++k) {
                if (h[k] == 0) {
                    // sweep k changed nothing, so it copied end_in to end_out and
                    // both buffers hold the converged ends; later sweeps exited early.
                    done = true;
                    break;
                }
                ++iters;
            }
            if (!done && iters >= j->comp_max_iters)
                return set_err(c, MM_ERR_STATE, "compressor did not converge in %d sweeps", iters);
        }
        c->job.comp_max_iters = iters;  // reported via mm_result
        RET(launch(c, "comp_record", comp_record_kernel, dim3(nbs, 3), dim3(256), 0, ca));
        RET(launch(c, "comp_tstart", comp_tstart_kernel, dim3(nb, 3), dim3(256), 0, ca));
        RET(launch(c, "comp_apply", comp_apply_kernel, dim3(nb), dim3(256), 0, ca));
        mix = q2;
    } else {
        c->job.comp_max_iters = 0;
    }
    c->mix = mix;
    c->staged = true;
    return MM_OK;
}

// ------------------------------------------------------------ K-weighting
static int kweight_energies(mm_ctx *c, const double *carry_in_host, double *seg_host, double *range_end_host) {
    const mm_job *j = &c->job;
    const int64_t G = c->G;
    const int T = j->tile;
    double *z4, *s4, *part, *seg, *init = nullptr, *lend;
    int64_t *part_seg, *bounds;
    RET(get_buf(c, "z4", (size_t)std::max<int64_t>(G, 1) * 4, &z4));
    RET(get_buf(c, "s4", (size_t)std::max<int64_t>(G, 1) * 4, &s4));
    RET(get_buf(c, "kw_part", (size_t)std::max<int64_t>(G, 1) * 2, &part));
    RET(get_buf(c, "kw_part_seg", (size_t)std::max<int64_t>(G, 1), &part_seg));
    RET(get_buf(c, "kw_seg", (size_t)j->n_segs, &seg));
    RET(get_buf(c, "kw_bounds", (size_t)j->n_segs + 1, &bounds));
    RET(get_buf(c, "kw_lend", 8, &lend));
    HIPCHK(c, hipMemcpyAsync(bounds, j->seg_bounds, (j->n_segs + 1) * sizeof(int64_t), hipMemcpyHostToDevice,
                             c->stream));
    if (carry_in_host) {
        RET(get_buf(c, "kw_init", 8, &init));
        HIPCHK(c, hipMemcpyAsync(init, carry_in_host, 4 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    }
    KwArgs ka{};
    ka.N_proc = j->frames_proc;
    ka.G = G;
    ka.T = T;
    ka.ch = j->channels;
    for (int s = 0; s < 2; ++s)
        for (int k = 0; k < 5; ++k) ka.sos[s][k] = j->kweight.sos[s][k];
    ka.mix = c->mix;
    ka.z_out = z4;
    ka.s_in = s4;
    ka.n_segs = j->n_segs;
    ka.seg_bounds = bounds;
    ka.part = part;
    ka.part_seg = part_seg;
    const unsigned nb = blocks_for(G, 256);
    RET(launch(c, "kw_pass1", kweight_kernel<false>, dim3(nb), dim3(256), 0, ka));
    RET(run_scan(c, "kw_scan", j->kweight, 4, 1, G, G, z4, s4, init, lend));
    if (range_end_host) {
        HIPCHK(c, hipMemcpyAsync(range_end_host, lend, 4 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return MM_OK;
    }
    RET(launch(c, "kw_pass2", kweight_kernel<true>, dim3(nb), dim3(256), 0, ka));
    RET(launch(c, "seg_reduce", seg_reduce_kernel, dim3(blocks_for(j->n_segs, 256)), dim3(256), 0, ka, seg));
    HIPCHK(c, hipMemcpyAsync(seg_host, seg, j->n_segs * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MM_OK;
}

// pyloudnorm 0.1.1 integrated_loudness gating (mono, G=1), restated.
extern "C" int mm_gate_loudness(const mm_job *j, const double *seg_energy, double *loudness) {
    if (!j || !seg_energy || !loudness) return MM_ERR_ARG;
    const int64_t nb = j->n_blocks;
    std::vector<double> z((size_t)nb), l((size_t)nb);
    const int64_t *B = j->seg_bounds;
    const int64_t S = j->n_segs;
    for (int64_t b = 0; b < nb; ++b) {
        int64_t s0 = std::lower_bound(B, B + S + 1, j->block_lo[b]) - B;
        int64_t s1 = std::lower_bound(B, B + S + 1, j->block_hi[b]) - B;
        double acc = 0.0;
        for (int64_t s = s0; s < s1 && s < S; ++s) acc += seg_energy[s];
        z[b] = j->block_scale * acc;
        l[b] = -0.691 + 10.0 * std::log10(z[b]);
    }
    double sum = 0.0;
    int64_t cnt = 0;
    for (int64_t b = 0; b < nb; ++b)
        if (l[b] >= -70.0) {
            sum += z[b];
            ++cnt;
        }
    double mean_abs = cnt ? sum / (double)cnt : NAN;
    double gamma_r = -0.691 + 10.0 * std::log10(mean_abs) - 10.0;
    sum = 0.0;
    cnt = 0;
    for (int64_t b = 0; b < nb; ++b)
        if (l[b] > gamma_r && l[b] > -70.0) {
            sum += z[b];
            ++cnt;
        }
    double zavg = cnt ? sum / (double)cnt : 0.0;  // np.nan_to_num(mean([])) == 0
    *loudness = -0.691 + 10.0 * std::log10(zavg);
    return MM_OK;
}

static int finalize(mm_ctx *c, double gain, int use_gain, void *d_out) {
    const mm_job *j = &c->job;
    if (c->G == 0) return MM_OK;
    FinArgs fa{};
    fa.N_proc = j->frames_proc;
    fa.G = c->G;
    fa.T = j->tile;
    fa.ch = j->channels;
    fa.out_kind = j->out_kind;
    fa.use_gain = use_gain;
    fa.gain = gain;
    fa.mix = c->mix;
    fa.out = d_out;
    const size_t lds = (size_t)FIN_TILES * (j->tile + 1) * sizeof(short2);
    return launch(c, "finalize", finalize_kernel, dim3(blocks_for(c->G, FIN_TILES)), dim3(256), lds, fa);
}

static int master_device(mm_ctx *c, const mm_job *j, const float *d_in, void *d_out, mm_result *res) {
    RET(stage_chunks(c, j, d_in));
    double L = NAN, gain = 1.0;
    int use_gain = 0;
    if (j->lufs_on) {
        std::vector<double> seg((size_t)j->n_segs);
        if (c->G > 0) RET(kweight_energies(c, nullptr, seg.data(), nullptr));
        RET(mm_gate_loudness(j, seg.data(), &L));
        gain = std::pow(10.0, (j->lufs_target - L) / 20.0);
        use_gain = 1;
    }
    RET(finalize(c, gain, use_gain, d_out));
    if (res) {
        res->loudness = L;
        res->gain_linear = gain;
        res->frames_out = j->frames_proc;
        res->comp_iters = c->job.comp_max_iters;
    }
    return MM_OK;
}

// =================================================================== C-ABI
extern "C" {

int mm_version(void) { return 1; }

int mm_create(int device, mm_ctx **out) {
    if (!out) return MM_ERR_ARG;
    *out = nullptr;
    mm_ctx *c = new mm_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) {
        delete c;
        return MM_ERR_HIP;
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return MM_ERR_HIP;
    }
    *out = c;
    return MM_OK;
}

int mm_destroy(mm_ctx *c) {
    if (!c) return MM_OK;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->comm) ncclCommDestroy(c->comm);
    resolve_events(c);
    for (auto e : c->free_events) hipEventDestroy(e);
    for (auto &kv : c->bufs)
        if (kv.second.p) hipFree(kv.second.p);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return MM_OK;
}

const char *mm_last_error(mm_ctx *c) { return c ? c->err : "null context"; }

int mm_sync(mm_ctx *c) {
    if (!c) return MM_ERR_ARG;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    return MM_OK;
}

int mm_master_device(mm_ctx *c, const mm_job *j, const float *d_in, void *d_out, mm_result *res) {
    if (!c) return MM_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    return master_device(c, j, d_in, d_out, res);
}

int mm_master(mm_ctx *c, const mm_job *j, const float *in, void *out, mm_result *res) {
    if (!c) return MM_ERR_ARG;
    RET(validate(c, j));
    HIPCHK(c, hipSetDevice(c->device));
    float *d_in;
    void *d_out;
    const size_t in_n = (size_t)j->frames_in * j->channels;
    const size_t out_bytes = (size_t)j->frames_proc * j->channels * (j->out_kind == MM_OUT_I16 ? 2 : 4);
    RET(get_buf(c, "host_in", std::max<size_t>(in_n, 1), &d_in));
    char *ob;
    RET(get_buf(c, "host_out", std::max<size_t>(out_bytes, 1), &ob));
    d_out = ob;
    if (in_n) HIPCHK(c, hipMemcpyAsync(d_in, in, in_n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    RET(master_device(c, j, d_in, d_out, res));
    if (out_bytes) HIPCHK(c, hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    return MM_OK;
}

int mm_stage_chunks(mm_ctx *c, const mm_job *j, const float *d_in) {
    if (!c) return MM_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    return stage_chunks(c, j, d_in);
}

int mm_kweight_range_end(mm_ctx *c, double *end_state_host) {
    if (!c || !c->staged) return set_err(c, MM_ERR_STATE, "no staged job");
    if (c->G == 0) {
        for (int k = 0; k < 4; ++k) end_state_host[k] = 0.0;
        return MM_OK;
    }
    return kweight_energies(c, nullptr, nullptr, end_state_host);
}

int mm_hop_energies(mm_ctx *c, const double *carry_in_host, double *seg_energy_host) {
    if (!c || !c->staged) return set_err(c, MM_ERR_STATE, "no staged job");
    if (c->G == 0) {
        for (int64_t s = 0; s < c->job.n_segs; ++s) seg_energy_host[s] = 0.0;
        return MM_OK;
    }
    return kweight_energies(c, carry_in_host, seg_energy_host, nullptr);
}

int mm_finalize(mm_ctx *c, double gain_linear, int use_gain, void *d_out) {
    if (!c || !c->staged) return set_err(c, MM_ERR_STATE, "no staged job");
    return finalize(c, gain_linear, use_gain, d_out);
}

int mm_read_mix(mm_ctx *c, int16_t *host_mix) {
    if (!c || !c->staged) return set_err(c, MM_ERR_STATE, "no staged job");
    const mm_job *j = &c->job;
    const int64_t N = j->frames_proc;
    if (N == 0) return MM_OK;
    int16_t *tmp;
    RET(get_buf(c, "mix_nat", (size_t)N * j->channels, &tmp));
    RET(launch(c, "mix_to_natural", mix_to_natural_kernel, dim3(blocks_for(N, 256)), dim3(256), 0,
               (const short2 *)c->mix, tmp, c->G, j->tile, N, j->channels));
    HIPCHK(c, hipMemcpyAsync(host_mix, tmp, (size_t)N * j->channels * sizeof(int16_t), hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MM_OK;
}

int mm_timing(mm_ctx *c, int enable) {
    if (!c) return MM_ERR_ARG;
    c->timing = enable != 0;
    if (!enable) {
        c->stats.clear();
        c->stat_order.clear();
    }
    return MM_OK;
}

int mm_kernel_stats(mm_ctx *c, char *names, int names_cap, double *total_ms, int64_t *launches, int cap) {
    if (!c) return MM_ERR_ARG;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    std::string joined;
    int n = 0;
    for (auto &nm : c->stat_order) {
        if (n >= cap) break;
        total_ms[n] = c->stats[nm].ms;
        launches[n] = c->stats[nm].n;
        if (n) joined += "\n";
        joined += nm;
        ++n;
    }
    if (names && names_cap > 0) {
        strncpy(names, joined.c_str(), (size_t)names_cap - 1);
        names[names_cap - 1] = 0;
    }
    return n;
}

int mm_comm_unique_id(char id_out[128]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return MM_ERR_RCCL;
    static_assert(sizeof(id) == 128, "nccl unique id size");
    memcpy(id_out, &id, 128);
    return MM_OK;
}

int mm_comm_init(mm_ctx *c, int rank, int nranks, const char id[128]) {
    if (!c) return MM_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId uid;
    memcpy(&uid, id, 128);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) return set_err(c, MM_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
    c->rank = rank;
    c->nranks = nranks;
    return MM_OK;
}

int mm_comm_destroy(mm_ctx *c) {
    if (!c) return MM_ERR_ARG;
    if (c->comm) ncclCommDestroy(c->comm);
    c->comm = nullptr;
    return MM_OK;
}

int mm_allreduce_sum_f64(mm_ctx *c, double *host_buf, int64_t n) {
    if (!c || !c->comm) return set_err(c, MM_ERR_STATE, "communicator not initialised");
    double *d;
    RET(get_buf(c, "coll", (size_t)std::max<int64_t>(n, 1), &d));
    HIPCHK(c, hipMemcpyAsync(d, host_buf, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    ncclResult_t r = ncclAllReduce(d, d, (size_t)n, ncclDouble, ncclSum, c->comm, c->stream);
    if (r != ncclSuccess) return set_err(c, MM_ERR_RCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
    HIPCHK(c, hipMemcpyAsync(host_buf, d, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MM_OK;
}

int mm_allgather_f64(mm_ctx *c, const double *host_in, double *host_out, int64_t n) {
    if (!c || !c->comm) return set_err(c, MM_ERR_STATE, "communicator not initialised");
    double *d;
    RET(get_buf(c, "coll_ag", (size_t)std::max<int64_t>(n * (c->nranks + 1), 1), &d));
    double *dout = d + n;
    HIPCHK(c, hipMemcpyAsync(d, host_in, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    ncclResult_t r = ncclAllGather(d, dout, (size_t)n, ncclDouble, c->comm, c->stream);
    if (r != ncclSuccess) return set_err(c, MM_ERR_RCCL, "ncclAllGather: %s", ncclGetErrorString(r));
    HIPCHK(c, hipMemcpyAsync(host_out, dout, n * c->nranks * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MM_OK;
}

}  // extern "C"
