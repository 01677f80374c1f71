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
#include "iir.hip"
#include "kernels.hip"
#include "compressor.hip"
#include "gate.hip"

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
    int n_cus = 256;  // compute units of the device (persistent launches)
    hipStream_t stream = nullptr;
    char err[512] = {0};
    std::map<std::string, DevBuf> bufs;
    // staged job geometry (mm_stage_chunks -> mm_hop_energies / mm_finalize)
    bool staged = false;
    mm_job job{};
    int64_t G = 0;
    short2 *mix = nullptr;
    unsigned *lb_error = nullptr;
    // per-chain control words, zeroed by ONE memset at the chain start: the three
    // IIR stages' ticket/status regions and the compressor's sweep flags; a
    // region is "fresh" until its first use (repeats zero their own words)
    unsigned *ctl_lb[3] = {nullptr, nullptr, nullptr};
    bool ctl_fresh[3] = {false, false, false};
    bool comp_flags_fresh = false;
    // compressor state kept across the queued launches (stage_front -> comp_sweeps/comp_back)
    bool comp_on = false;
    CompArgs ca{};
    uint32_t comp_stamp = 0;  // stamp of the last queued fix-up sweep
    unsigned *comp_changed = nullptr;
    char *ctl = nullptr;                // the chain's control block (setup_control)
    size_t ctl_bytes = 0, ctl_rba = 0;  // its size and readback area
    // the block is zero from ctl_clean_ptr up to ctl_clean_bytes: the last chain's
    // tail (finalize) zeroed it, so the next setup_control queues no fill
    bool ctl_clean = false;
    char *ctl_clean_ptr = nullptr;
    size_t ctl_clean_bytes = 0;
    bool tail_readback = false;         // the last queued finalize hands the readback area over
    uint32_t *ctl_claims = nullptr;     // its zeroed claim stamps
    int comp_iters = 0, comp_pending = 0;
    int comp_queue = 0;  // sweeps to queue with the next solve (0: COMP_SWEEPS; then the last solve's need + 1)
    uint64_t comp_sig = 0;  // settings and geometry of the solve comp_queue was learnt on (comp_signature)
    // loudness on the device
    double *gate_out = nullptr;         // [2]: L, gain
    std::vector<int64_t> geom_cache;    // loudness geometry already on the device
    int32_t *blk_s0 = nullptr, *blk_s1 = nullptr;
    int64_t *seg_bounds_dev = nullptr;
    // exact block energies (kw_blocks_kernel): per block its first frame and program
    int64_t *kb_lo = nullptr;
    int32_t *kb_n = nullptr, *kb_prog_of = nullptr, *kb_prog = nullptr;
    std::vector<int64_t> kb_cache;      // block geometry the programs on the device were built for
    int kb_nvals = 0, kb_pints = 0;     // the largest program's values and ints (kw_blocks' LDS)
    // timing
    bool timing = false;
    std::vector<PendingEvent> pending;
    std::vector<hipEvent_t> free_events;
    // pinned double-buffered staging for the WAV file path (mm_master_wav)
    char *pin[2] = {nullptr, nullptr};
    hipEvent_t pin_ev[2] = {nullptr, nullptr};
    std::map<std::string, KStat> stats;
    std::vector<std::string> stat_order;
    // host tables already resident on the device
    uint64_t lut_key[3] = {0, 0, 0};  // content keys of the band tables on the device (0: none)
    uint64_t sat_key = 0;             // content key of the exciter table on the device (0: none)
    bool sat_codes = false;           // its correction codes are complete (no entry needs the table)
    std::map<std::string, std::vector<double>> mats_cache;
    // pinned block the chain's results are copied into (one sync per chain)
    char *rb = nullptr, *rb_dev = nullptr;  // (rb_dev: its device address)
    size_t rb_cap = 0;
    // batch execution (mm_master_batch): child contexts, one stream each
    std::vector<mm_ctx *> children;
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

#define RET_EARLY(expr)             \
    do {                            \
        int r_ = (expr);            \
        if (r_ != MM_OK) return r_; \
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

// ------------------------------------------------------- look-back plumbing
// Transition tables of one filter stage (uploaded only when they change).
static int upload_tables(mm_ctx *c, const char *name, const mm_iir &f, LbArgs &lb) {
    const size_t n = (size_t)(MM_TILE_POW + MM_BLK_POW) * 64;
    std::vector<double> host(n);
    memcpy(host.data(), f.phi_tile_pow, sizeof f.phi_tile_pow);
    memcpy(host.data() + MM_TILE_POW * 64, f.phi_blk_pow, sizeof f.phi_blk_pow);
    const std::string key = std::string("tab_") + name;
    double *d;
    RET(get_buf(c, key.c_str(), n, &d));
    std::vector<double> &cached = c->mats_cache[key];
    if (cached != host) {
        HIPCHK(c, hipMemcpyAsync(d, host.data(), n * sizeof(double), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));  // host vector is transient
        cached = host;
    }
    lb.pw_tile = d;
    lb.pw_blk = d + MM_TILE_POW * 64;
    return MM_OK;
}

// Zero-state weights of one stage over a whole tile of T frames (pass 1 of the
// crossover as a product, XoArgs::zw): row n is the state after the tile from a
// zero state with a unit input at frame n and zeros elsewhere, W[n] = A^(T-1-n) B
// (A: one zero-input frame, B: the state one frame after a unit input), evaluated
// in long double and rounded once.  Branch 0 is sections [0, nsec_branch0), branch 1
// the rest, both fed by the stage input (csrc/lookback.h's layout).
static void zs_weights(const mm_iir &f, int T, std::vector<double> &W) {
    const int nsec = f.nsec, nb0 = f.nsec_branch0;
    auto step = [&](const long double *z, long double x, long double *o) {
        for (int br = 0; br < 2; ++br) {
            long double u = x;
            for (int s = br ? nb0 : 0; s < (br ? nsec : nb0); ++s) {
                const double *c = f.sos[s];
                const long double y = (long double)c[0] * u + z[2 * s];
                o[2 * s] = (long double)c[1] * u - (long double)c[3] * y + z[2 * s + 1];
                o[2 * s + 1] = (long double)c[2] * u - (long double)c[4] * y;
                u = y;
            }
        }
    };
    W.assign((size_t)T * 8, 0.0);
    long double v[8] = {0}, t[8] = {0}, zero[8] = {0};
    step(zero, 1.0L, v);
    for (int n = T - 1; n >= 0; --n) {
        for (int d = 0; d < 2 * nsec; ++d) W[(size_t)n * 8 + d] = (double)v[d];
        step(v, 0.0L, t);
        for (int d = 0; d < 8; ++d) v[d] = t[d];
    }
}

// The stage's zero-state weights on the device (rebuilt only when its sections or
// the tile change); null with MM_ZS_RECUR (A/B: pass 1 as the recurrence).
static int upload_zw(mm_ctx *c, const char *name, const mm_iir &f, int T, const double **out) {
    static const bool recur = getenv("MM_ZS_RECUR") != nullptr;
    *out = nullptr;
    if (recur || f.nsec < 1 || f.nsec > 4) return MM_OK;
    std::vector<double> key(f.sos[0], f.sos[0] + 20);
    key.push_back((double)T);
    key.push_back((double)f.nsec);
    key.push_back((double)f.nsec_branch0);
    const std::string kname = std::string("zw_") + name;
    double *d;
    RET(get_buf(c, kname.c_str(), (size_t)T * 8, &d));
    std::vector<double> &cached = c->mats_cache[kname];
    if (cached != key) {
        std::vector<double> W;
        zs_weights(f, T, W);
        HIPCHK(c, hipMemcpyAsync(d, W.data(), W.size() * sizeof(double), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));  // host vector is transient
        cached = key;
    }
    *out = d;
    return MM_OK;
}

// Per-launch look-back state for nblk blocks of CH lines: the ticket and the
// status words are zeroed by a memset on the stream right before the launch.
static size_t lb_flag_bytes(int64_t nblk) { return ((16 + (size_t)nblk * 4) + 15) / 16 * 16; }

// region: the chain's pre-zeroed control region of this stage (0 eq, 1 crossover,
// 2 K-weighting), used once; otherwise (or on a repeat) a private memset.
static int lb_prepare(mm_ctx *c, int64_t nblk, int ch, LbArgs &lb, int region = -1) {
    char *flags;
    if (region >= 0 && c->ctl_fresh[region]) {
        flags = reinterpret_cast<char *>(c->ctl_lb[region]);
        c->ctl_fresh[region] = false;
    } else {
        const size_t flag_bytes = lb_flag_bytes(nblk);
        RET(get_buf(c, "lb_flags", flag_bytes, &flags));
        HIPCHK(c, hipMemsetAsync(flags, 0, flag_bytes, c->stream));
    }
    lb.ticket = reinterpret_cast<unsigned *>(flags);
    lb.status = reinterpret_cast<unsigned *>(flags + 16);
    RET(get_buf(c, "lb_agg", (size_t)nblk * ch * 8, &lb.agg));
    RET(get_buf(c, "lb_incl", (size_t)nblk * ch * 8, &lb.incl));
    if (c->lb_error) lb.error = c->lb_error;
    else RET(get_buf(c, "lb_error", 4, &lb.error));
    lb.init = nullptr;
    return MM_OK;
}

static int validate(mm_ctx *c, const mm_job *j) {
    if (!j) return set_err(c, MM_ERR_ARG, "null job");
    if (j->channels != 1 && j->channels != 2) return set_err(c, MM_ERR_ARG, "channels must be 1 or 2");
    if (j->in_kind != MM_IN_F32 && j->in_kind != MM_IN_I16) return set_err(c, MM_ERR_ARG, "in_kind %d", j->in_kind);
    if (j->tile < 16 || j->tile > 512) return set_err(c, MM_ERR_ARG, "tile %d out of range [16, 512]", j->tile);
    if (j->tiles_per_chunk < 1) return set_err(c, MM_ERR_ARG, "tiles_per_chunk < 1");
    if (j->frames_proc < 0 || j->frames_in < 0) return set_err(c, MM_ERR_ARG, "negative frame count");
    if (j->frames_proc >= (int64_t)1 << 31 || j->frames_in >= (int64_t)1 << 31)
        return set_err(c, MM_ERR_ARG, "track longer than 2^31 frames (32-bit frame indexing)");
    if (j->eq.nsec < 0 || j->eq.nsec > 4) return set_err(c, MM_ERR_ARG, "eq.nsec %d", j->eq.nsec);
    const int tpb = LB_THREADS / j->channels;
    if (j->eq.nsec > 0 && j->eq.tpb != tpb) return set_err(c, MM_ERR_ARG, "eq tables built for %d tiles/block, need %d", j->eq.tpb, tpb);
    if (j->multiband_on && j->xover.tpb != tpb) return set_err(c, MM_ERR_ARG, "crossover tables built for %d tiles/block", j->xover.tpb);
    if (j->lufs_on && j->kweight.tpb != LB_THREADS) return set_err(c, MM_ERR_ARG, "K-weighting tables built for %d tiles/block", j->kweight.tpb);
    if (j->eq.nsec > 0 && j->eq.tile != j->tile) return set_err(c, MM_ERR_ARG, "eq tables built for %d-frame tiles", j->eq.tile);
    if (j->multiband_on && j->xover.tile != j->tile) return set_err(c, MM_ERR_ARG, "crossover tables built for %d-frame tiles", j->xover.tile);
    if (j->lufs_on && (j->kweight.tile < 1 || j->tile % j->kweight.tile != 0))
        return set_err(c, MM_ERR_ARG, "K-weighting tables built for %d-frame (sub-)tiles, not a divisor of %d",
                       j->kweight.tile, j->tile);
    if (j->multiband_on) {
        if (j->xover.nsec != 4 || j->xover.nsec_branch0 != 2) return set_err(c, MM_ERR_ARG, "crossover must be 2+2 sections");
        for (int b = 0; b < 3; ++b) {
            if (!j->band[b].lut) return set_err(c, MM_ERR_ARG, "band %d: missing table", b);
            if (j->band[b].look < 0) return set_err(c, MM_ERR_ARG, "band %d: look < 0", b);
            if (!(j->band[b].release_frames >= 1.0) || !(j->band[b].attack_frames > 0.0))
                return set_err(c, MM_ERR_ARG, "band %d: release must span >= 1 frame", b);
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

template <int NS>
static int launch_eq_ns(mm_ctx *c, int ch, unsigned nblk, const EqArgs &ea, const LbArgs &lb, int64_t K) {
    if (ch == 2) {
        const size_t lds = eq_lds_bytes<NS, 2>();
        if (ea.in16) return launch(c, "eq", eq_kernel<NS, 2, true>, dim3(nblk), dim3(LB_THREADS), lds, ea, lb, K);
        return launch(c, "eq", eq_kernel<NS, 2, false>, dim3(nblk), dim3(LB_THREADS), lds, ea, lb, K);
    }
    const size_t lds = eq_lds_bytes<NS, 1>();
    if (ea.in16) return launch(c, "eq", eq_kernel<NS, 1, true>, dim3(nblk), dim3(LB_THREADS), lds, ea, lb, K);
    return launch(c, "eq", eq_kernel<NS, 1, false>, dim3(nblk), dim3(LB_THREADS), lds, ea, lb, K);
}

static int launch_eq(mm_ctx *c, int nsec, int ch, unsigned nblk, const EqArgs &ea, const LbArgs &lb, int64_t K) {
    switch (nsec) {
        case 1: return launch_eq_ns<1>(c, ch, nblk, ea, lb, K);
        case 2: return launch_eq_ns<2>(c, ch, nblk, ea, lb, K);
        case 3: return launch_eq_ns<3>(c, ch, nblk, ea, lb, K);
        default: return launch_eq_ns<4>(c, ch, nblk, ea, lb, K);
    }
}

// --------------------------------------------------- compressor sweeps
// Fix-up sweeps are queued without a host sync: sweep k writes flag k (some
// successor may be stale) and exits at once if sweep k-1 flagged nothing.
// Convergence is checked at the chain's single sync (evaluate_chain); a rare
// unconverged batch is extended there (MM_COMP_SWEEPS sets the queued count).
constexpr int COMP_SWEEPS = 8;  // queued by a context's first solve (a sweep after a quiet one exits at once)

static int comp_sweeps(mm_ctx *c, int n) {
    CompArgs &ca = c->ca;
    const int64_t NS = ca.GS;
    if (!c->comp_flags_fresh)  // flags only (the walked count accumulates)
        HIPCHK(c, hipMemsetAsync(c->comp_changed, 0, 16 * sizeof(unsigned int), c->stream));
    c->comp_flags_fresh = false;
    for (int k = 0; k < n; ++k) {
        ca.sweep_idx = (int)c->comp_stamp;
        ca.stamp = ++c->comp_stamp;
        ca.heads = ca.stamp > 1 ? 1 : 0;  // the chain's first sweep is a Jacobi step
        ca.changed = c->comp_changed + k;
        const unsigned int *prevf = k > 0 ? c->comp_changed + (k - 1) : nullptr;
        RET(launch(c, "comp_fix", comp_fix_kernel, dim3(blocks_for(NS, 64), 3), dim3(64), 0, ca, prevf));
    }
    c->comp_pending = n;
    return MM_OK;
}

// gains + overlay into q2, every tile starting from its stored entry state
static int comp_back(mm_ctx *c) {
    const CompArgs &ca = c->ca;
    const int64_t nchunks = ca.GS / ca.SPC;  // (chunk-aligned blocks of APPLY_TILES tiles)
    return launch(c, "comp_apply", comp_apply_kernel,
                  dim3((unsigned)(nchunks * ((ca.K + APPLY_TILES - 1) / APPLY_TILES))), dim3(3 * APPLY_TILES), 0, ca);
}

// Pinned readback block of one chain pass (offsets in bytes): look-back error
// word, sweep flags, re-walked frame count, loudness + gain, per-chunk active counts.
constexpr size_t RB_ERR = 0, RB_FLAGS = 16, RB_WALKED = 80, RB_LG = 96, RB_TOTALS = 128;
// finalize's done counters after the readback area (FIN_DONE_LINES lines of 128 B and
// the top one; FinArgs::done)
constexpr size_t FIN_DONE_BYTES = (size_t)(FIN_DONE_LINES + 1) * 128;
static size_t rb_bytes(int64_t nch) { return RB_TOTALS + (size_t)12 * nch; }

static int64_t comp_chunks(const mm_ctx *c) { return c->comp_on ? c->ca.GS / c->ca.SPC : 0; }

static int ensure_rb(mm_ctx *c, size_t bytes) {
    if (c->rb_cap >= bytes) return MM_OK;
    if (c->rb) HIPCHK(c, hipHostFree(c->rb));
    c->rb = c->rb_dev = nullptr;
    c->rb_cap = 0;
    // mapped and coherent: the chain's last finalize block writes it directly
    HIPCHK(c, hipHostMalloc((void **)&c->rb, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(c, hipHostGetDevicePointer((void **)&c->rb_dev, c->rb, 0));
    c->rb_cap = bytes;
    return MM_OK;
}

// Hand the readback area over in the chain's last finalize launch (FinArgs::ctl),
// instead of a copy after it.
static int attach_tail(mm_ctx *c, FinArgs &fa) {
    static const bool off = getenv("MM_CTL_FILL") != nullptr;  // (A/B: the round-5 fill + copy)
    c->tail_readback = false;
    if (off || !c->ctl) return MM_OK;
    const size_t rbb = rb_bytes(comp_chunks(c));
    RET(ensure_rb(c, rbb + 64));
    fa.ctl = c->ctl;
    fa.ctl_bytes = (int64_t)c->ctl_bytes;
    fa.rb_area = (int64_t)(c->ctl_rba + FIN_DONE_BYTES);
    fa.rb_bytes = (int)rbb;
    fa.rb_host = c->rb_dev;
    fa.done = reinterpret_cast<unsigned *>(c->ctl + c->ctl_rba);
    c->tail_readback = true;
    return MM_OK;
}

// Queue the D2H copy of everything the host checks after the chain (no sync): the
// readback area of the control block, in ONE copy.
static int queue_readback(mm_ctx *c, bool lufs) {
    (void)lufs;
    const int64_t nch = comp_chunks(c);
    RET(ensure_rb(c, rb_bytes(nch) + 64));
    HIPCHK(c, hipMemcpyAsync(c->rb, c->ctl, rb_bytes(nch), hipMemcpyDeviceToHost, c->stream));
    return MM_OK;
}

// After the stream has drained: reports look-back timeouts (never expected: a
// block only waits on blocks that started before it) and whether the queued
// sweeps converged.
static int evaluate_chain(mm_ctx *c, bool *converged) {
    static const bool debug_walked = getenv("MM_DEBUG_WALKED") != nullptr;
    if (debug_walked)
        fprintf(stderr, "walked=%llu jumped=%llu\n", *reinterpret_cast<const unsigned long long *>(c->rb + RB_WALKED),
                *reinterpret_cast<const unsigned long long *>(c->rb + RB_WALKED + 8));
    if (*reinterpret_cast<const unsigned *>(c->rb + RB_ERR)) return set_err(c, MM_ERR_STATE, "IIR look-back timed out");
    if (c->comp_on && c->ca.trace) {  // MM_FIX_TRACE: the three slowest walkers of every sweep
        const int64_t NS = c->ca.GS;
        std::vector<uint32_t> tr((size_t)16 * 3 * NS * 4);
        HIPCHK(c, hipMemcpy(tr.data(), c->ca.trace, tr.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (const char *path = getenv("MM_FIX_TRACE_DUMP")) {  // every walker record: [sweep][band][super-tile][4]
            if (FILE *f = fopen(path, "wb")) {
                fwrite(tr.data(), sizeof(uint32_t), tr.size(), f);
                fclose(f);
            }
        }
        for (int k = 0; k < 16; ++k) {
            std::vector<std::pair<uint32_t, int64_t>> v;
            int64_t nw = 0;
            for (int64_t i = 0; i < 3 * NS; ++i) {
                const uint32_t *r = &tr[((size_t)k * 3 * NS + i) * 4];
                if (r[0] || r[3]) {
                    v.push_back({r[0], i});
                    ++nw;
                }
            }
            if (v.empty()) continue;
            std::sort(v.rbegin(), v.rend());
            fprintf(stderr, "sweep %d: %lld walkers;", k, (long long)nw);
            for (size_t q = 0; q < std::min<size_t>(3, v.size()); ++q) {
                const uint32_t *r = &tr[((size_t)k * 3 * NS + v[q].second) * 4];
                fprintf(stderr, " [band %lld st %lld: %.1f us walked %u jumped %u visited %u]",
                        (long long)(v[q].second / NS), (long long)(v[q].second % NS), r[0] / 100.0, r[1], r[2],
                        r[3]);
            }
            fprintf(stderr, "\n");
        }
    }
    *converged = true;
    if (c->comp_on && c->comp_pending) {
        const unsigned *flags = reinterpret_cast<const unsigned *>(c->rb + RB_FLAGS);
        int k = 0;
        while (k < c->comp_pending && flags[k]) ++k;
        c->comp_iters += k;
        *converged = k < c->comp_pending;
        c->comp_pending = 0;
        // the solve needed comp_iters flagged sweeps and one quiet one: queue that + 1
        if (*converged) c->comp_queue = std::min(16, std::max(3, c->comp_iters + 2));
        if (!*converged && c->comp_iters >= c->job.comp_max_iters)
            return set_err(c, MM_ERR_STATE, "compressor did not converge in %d sweeps", c->comp_iters);
    }
    return MM_OK;
}

// An extension after a tail hand-over starts from a zeroed control block: the
// per-chunk active counts (comp_rms, once per chain) and the earlier passes'
// re-walked counts are kept on the host and merged into the last readback.
struct RbKeep {
    bool on = false;
    std::vector<int32_t> tot;
    unsigned long long walked[2] = {0, 0};
};
static void rb_keep(mm_ctx *c, RbKeep &k) {
    if (!c->tail_readback) return;  // (a copied readback: the device words accumulate)
    const int32_t *tot = reinterpret_cast<const int32_t *>(c->rb + RB_TOTALS);
    if (!k.on) k.tot.assign(tot, tot + 3 * comp_chunks(c));
    const unsigned long long *w = reinterpret_cast<const unsigned long long *>(c->rb + RB_WALKED);
    k.walked[0] += w[0];
    k.walked[1] += w[1];
    k.on = true;
    c->comp_flags_fresh = true;  // the sweep flags are zero as well
}
// After the chain's last pass: merge what rb_keep held, and note a zeroed block.
static void rb_finish(mm_ctx *c, const RbKeep &k) {
    if (k.on) {
        memcpy(c->rb + RB_TOTALS, k.tot.data(), k.tot.size() * sizeof(int32_t));
        unsigned long long *w = reinterpret_cast<unsigned long long *>(c->rb + RB_WALKED);
        w[0] += k.walked[0];
        w[1] += k.walked[1];
    }
    c->ctl_clean = c->tail_readback;
    c->ctl_clean_ptr = c->ctl;
    c->ctl_clean_bytes = c->ctl_bytes;
}

static int chain_check(mm_ctx *c, bool *converged) {
    RET(queue_readback(c, false));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return evaluate_chain(c, converged);
}

// Geometry of the envelope solve (the C-ABI's mm_solve_geometry): TPS tiles per
// super-tile (the job's comp_super frames rounded to whole tiles), columns per
// chunk in whole blocks of 64 (comp_rms stores; a wave's columns lie in one
// chunk), plane rows per tile and per column, and each chunk's own plane (32-bit
// buffer offsets within it at any track length).
static int solve_geometry(const mm_job *j, mm_solve_geom *g) {
    const int K = j->tiles_per_chunk, T = j->tile;
    if (K < 1 || T < 1 || j->frames_proc < 0) return MM_ERR_ARG;
    const int64_t G = (j->frames_proc + T - 1) / T;
    *g = mm_solve_geom{};
    g->tps = std::max(1, std::min((j->comp_super + T / 2) / T, DESC_MAX_TPS));  // (comp_describe: 64 TPS threads)
    if (g->tps != RMS_TPS) return MM_ERR_ARG;  // comp_rms_t's workgroup: RMS_TPS positions x 64 columns
    g->col_block = 64;
    g->rms_group_tiles = RMS_TPS * 64;
    g->chunks = (G + K - 1) / K;
    g->cols_per_chunk = (((int64_t)K + g->tps - 1) / g->tps + 63) / 64 * 64;
    g->walk_block = WB;
    g->tile_rows = (T + WB - 1) / WB * WB;
    g->rows = g->tps * g->tile_rows + WALK_PAD;
    g->chunk_plane_bytes = (int64_t)g->rows * g->cols_per_chunk * 8;
    g->plane_bytes = 3 * g->chunks * g->chunk_plane_bytes;
    return g->chunk_plane_bytes < ((int64_t)1 << 31) ? MM_OK : MM_ERR_ARG;
}

// Control words of the whole chain: the readback area (RB_* layout: look-back
// error word, sweep flags, re-walked count, loudness + gain, per-chunk active
// counts), finalize's done counters, the sweeps' claim stamps, then the eq /
// crossover / K-weighting look-back regions (each fresh until its first use).  The chain's
// last finalize hands the readback area to the mapped host block and leaves the
// whole block zeroed (FinArgs::ctl), so a chain after a completed one starts with
// no fill and ends with no copy; otherwise ONE memset here and ONE copy at the end.
static int setup_control(mm_ctx *c, unsigned nblk, int64_t nch, int64_t claims) {
    const size_t region = lb_flag_bytes(nblk);  // >= the K-weighting stage's (256 tiles per block)
    const size_t rba = (rb_bytes(nch) + 255) / 256 * 256, cla = ((size_t)claims * 4 + 255) / 256 * 256;
    const size_t bytes = rba + FIN_DONE_BYTES + cla + 3 * region;
    char *ctl;
    RET(get_buf(c, "ctl", bytes, &ctl));
    static const bool always_fill = getenv("MM_CTL_FILL") != nullptr;  // (A/B: round 5's fill per chain)
    if (always_fill || !c->ctl_clean || ctl != c->ctl_clean_ptr || bytes > c->ctl_clean_bytes)
        HIPCHK(c, hipMemsetAsync(ctl, 0, bytes, c->stream));
    c->ctl_clean = false;
    c->ctl = ctl;
    c->ctl_bytes = bytes;
    c->ctl_rba = rba;
    c->lb_error = reinterpret_cast<unsigned *>(ctl + RB_ERR);
    c->comp_changed = reinterpret_cast<unsigned *>(ctl + RB_FLAGS);
    c->gate_out = reinterpret_cast<double *>(ctl + RB_LG);
    c->ctl_claims = reinterpret_cast<uint32_t *>(ctl + rba + FIN_DONE_BYTES);
    for (int r = 0; r < 3; ++r) {
        c->ctl_lb[r] = reinterpret_cast<unsigned *>(ctl + rba + FIN_DONE_BYTES + cla + r * region);
        c->ctl_fresh[r] = true;
    }
    c->comp_flags_fresh = true;
    return MM_OK;
}

// Stage C (AME:207-210): per-band pydub compressor envelope solve + gains +
// overlay of the three int16 band planes (tile-major) into q2.  tile_e holds the
// crossover's per-tile band energies ([3][E, tail][G]).  Queues everything up to
// the apply; convergence is checked at the chain's sync.
// FNV-1a over the job fields the envelope solve's sweep count depends on
static uint64_t comp_signature(const mm_job *j) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](const void *p, size_t n) {
        const unsigned char *b = static_cast<const unsigned char *>(p);
        for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    };
    mix(&j->frames_proc, sizeof j->frames_proc);
    mix(&j->rate, sizeof j->rate);
    mix(&j->tile, sizeof j->tile);
    mix(&j->tiles_per_chunk, sizeof j->tiles_per_chunk);
    mix(&j->comp_super, sizeof j->comp_super);
    for (const mm_band &b : j->band) {
        mix(&b.thresh_rms, sizeof b.thresh_rms);
        mix(&b.attack_frames, sizeof b.attack_frames);
        mix(&b.release_frames, sizeof b.release_frames);
        mix(&b.look, sizeof b.look);
        mix(&b.r0, sizeof b.r0);
        mix(&b.lut_key, sizeof b.lut_key);
    }
    return h;
}

static int stage_compress(mm_ctx *c, const mm_job *j, short2 *const bands[3], const double *tile_e, short2 **q2_out) {
    const int T = j->tile, ch = j->channels, K = j->tiles_per_chunk;
    const int64_t N = j->frames_proc;
    const int64_t G = c->G;
    const int64_t TG = (int64_t)T * std::max<int64_t>(G, 1);
    CompArgs ca{};
    ca.N_proc = N;
    ca.G = G;
    ca.T = T;
    ca.K = K;
    ca.ch = ch;
    ca.warmup = j->comp_warmup;
    mm_solve_geom sg;
    if (solve_geometry(j, &sg) != MM_OK)
        return set_err(c, MM_ERR_ARG, "chunk of %d tiles too large for one envelope-solve plane", K);
    const int64_t nchunks = sg.chunks;
    ca.TPS = sg.tps;
    ca.SPC = sg.cols_per_chunk;
    ca.GS = nchunks * ca.SPC;
    const int64_t NS = ca.GS;
    short2 *q2;
    RET(get_buf(c, "q2", TG, &q2));
    ca.q_out = q2;
    *q2_out = q2;
    double *st, *ends, *luts, *tstc, *descc, *mmax, *mmaxc, *ced, *cedc;
    uint32_t *claims;
    RET(get_buf(c, "comp_start", (size_t)3 * NS, &st));
    RET(get_buf(c, "comp_end", (size_t)3 * NS, &ends));
    claims = c->ctl_claims;  // zeroed with the control block (sized by stage_front: claims, then cbtot)
    RET(get_buf(c, "comp_lut", (size_t)3 * 32769, &luts));
    const int64_t NC = nchunks * K;  // compact indices
    RET(get_buf(c, "comp_mmax", (size_t)3 * G, &mmax));
    RET(get_buf(c, "comp_tstc", (size_t)3 * NC, &tstc));
    RET(get_buf(c, "comp_mmaxc", (size_t)3 * NC, &mmaxc));
    RET(get_buf(c, "comp_ced", (size_t)6 * G, &ced));
    RET(get_buf(c, "comp_cedc", (size_t)6 * NC, &cedc));
    RET(get_buf(c, "comp_descc", (size_t)3 * DREC * NC, &descc));
    int32_t *ranks, *tls, *nacts;
    RET(get_buf(c, "comp_rank", (size_t)3 * G, &ranks));
    RET(get_buf(c, "comp_tl", (size_t)3 * NC, &tls));
    RET(get_buf(c, "comp_nact", (size_t)3 * nchunks, &nacts));
    ca.jumps = getenv("MM_COMP_NOJUMP") ? 0 : 1;  // diagnostics: results must not change
    ca.sjump = ca.jumps && !getenv("MM_COMP_NOSJUMP") && ca.TPS == SJ_TPS ? 1 : 0;
    ca.jacobi_stop = getenv("MM_JACOBI_STOP") ? 1 : 0;  // (tuning experiments)
    ca.e_tiles = E_TILES;
    if (const char *e = getenv("MM_E_TILES")) ca.e_tiles = std::max(0, atoi(e));  // (tuning experiments)
    double *sdesc;
    int32_t *se0s;
    RET(get_buf(c, "comp_sdesc", ca.sjump ? (size_t)3 * NS * SREC : 1, &sdesc));
    RET(get_buf(c, "comp_se0", ca.sjump ? (size_t)3 * NS : 1, &se0s));
    unsigned int *changed = c->comp_changed;  // zeroed with the chain's control words
    ca.walked = reinterpret_cast<unsigned long long *>(c->ctl + RB_WALKED);
    ca.trace = nullptr;
    if (getenv("MM_FIX_TRACE")) {  // diagnostics: per-walker sweep records, printed by evaluate_chain
        RET(get_buf(c, "comp_trace", (size_t)16 * 3 * NS * 4, &ca.trace));
        HIPCHK(c, hipMemsetAsync(ca.trace, 0, (size_t)16 * 3 * NS * 4 * sizeof(uint32_t), c->stream));
    }
    ca.TP = sg.tile_rows;
    ca.RP = sg.rows;
    ca.chunk_elems = sg.chunk_plane_bytes / 8;  // SPC / 64 column blocks of 64 x RP
    const int64_t ms_elems = ca.chunk_elems * nchunks;
    int32_t *cnt, *tot;
    RET(get_buf(c, "comp_cnt", (size_t)3 * G, &cnt));
    tot = reinterpret_cast<int32_t *>(c->ctl + RB_TOTALS);  // zeroed and read back with the control block
    for (int b = 0; b < 3; ++b) {
        double *msb;
        char nm[16];
        snprintf(nm, sizeof nm, "comp_ms%d", b);
        RET(get_buf(c, nm, (size_t)ms_elems, &msb));
        ca.Ms[b] = msb;
        ca.E[b] = tile_e + (size_t)(2 * b) * G;
        ca.tail[b] = tile_e + (size_t)(2 * b + 1) * G;
        ca.band[b] = bands[b];
        ca.lut[b] = luts + (size_t)b * 32769;
        // cached by content key (a host pointer may be reused by another table once the
        // caller frees one): upload when the key differs or is unknown
        if (j->band[b].lut_key == 0 || c->lut_key[b] != j->band[b].lut_key) {
            // the M column of the host's {M, M/A, M/R, 0} rows
            HIPCHK(c, hipMemcpy2DAsync(luts + (size_t)b * 32769, sizeof(double), j->band[b].lut,
                                       4 * sizeof(double), sizeof(double), 32769, hipMemcpyHostToDevice,
                                       c->stream));
            c->lut_key[b] = j->band[b].lut_key;
        }
        ca.r0[b] = (uint32_t)j->band[b].r0;
        ca.look[b] = j->band[b].look;
        ca.attack_frames[b] = j->band[b].attack_frames;
        ca.release_frames[b] = j->band[b].release_frames;
        ca.rcp_attack[b] = 1.0 / j->band[b].attack_frames;
        ca.rcp_release[b] = 1.0 / j->band[b].release_frames;
        ca.cnt[b] = cnt + (size_t)b * G;
        ca.mmax[b] = mmax + (size_t)b * G;
        ca.total[b] = tot + (size_t)b * nchunks;
        ca.rank[b] = ranks + (size_t)b * G;
        ca.nact[b] = nacts + (size_t)b * nchunks;
        ca.tl[b] = tls + (size_t)b * NC;
        ca.mmaxc[b] = mmaxc + (size_t)b * NC;
        ca.ced[b] = ced + (size_t)2 * b * G;
        ca.cedc[b] = cedc + (size_t)2 * b * NC;
        ca.tstc[b] = tstc + (size_t)b * NC;
        ca.descc[b] = descc + (size_t)b * DREC * NC;
        ca.start[b] = st + (size_t)b * NS;
        ca.end[b] = ends + (size_t)b * NS;
        ca.claim[b] = claims + (size_t)b * NS;
        ca.sdesc[b] = ca.sjump ? sdesc + (size_t)b * NS * SREC : nullptr;
        ca.se0[b] = ca.sjump ? se0s + (size_t)b * NS : nullptr;
        ca.cbtot[b] = reinterpret_cast<int32_t *>(claims + (size_t)3 * NS) + (size_t)b * (NS / 64);
    }
    // column block = one workgroup (RMS_TPS x 64 tiles): gathers / stores through LDS
    RET(launch(c, "comp_rms", comp_rms_t_kernel, dim3((unsigned)(NS / 64), 3), dim3(256), 0, ca));
    RET(launch(c, "comp_describe", comp_describe_kernel, dim3((unsigned)(NS / 64), 3), dim3(64 * ca.TPS), 0, ca));
    RET(launch(c, "comp_pass0", comp_pass0_kernel, dim3(blocks_for(NS, PASS0_BLOCK), 3), dim3(PASS0_BLOCK), 0, ca));
    c->comp_on = true;
    c->ca = ca;
    c->comp_stamp = 0;
    c->comp_changed = changed;
    c->comp_iters = 0;
    c->comp_pending = 0;
    // as many as the last solve on this context needed (+ 1 spare) when this job has
    // the same compressor settings and geometry: a stream of similar jobs queues few
    // idle sweeps and rarely resumes from the host; a job with other settings or
    // another length starts from COMP_SWEEPS again (a P_HOT job after P_FULL ones
    // would otherwise resume from the host)
    const uint64_t sig = comp_signature(j);
    if (sig != c->comp_sig) {
        c->comp_queue = 0;
        c->comp_sig = sig;
    }
    int sweeps = c->comp_queue > 0 ? c->comp_queue : COMP_SWEEPS;
    if (const char *e = getenv("MM_COMP_SWEEPS")) sweeps = std::max(1, std::min(16, atoi(e)));  // tests / tuning
    RET(comp_sweeps(c, sweeps));
    RET(comp_back(c));
    return MM_OK;
}

// ------------------------------------------------------------ chain A..C
static int stage_front(mm_ctx *c, const mm_job *j, const void *d_in) {
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
    const int tpb = LB_THREADS / ch;
    const unsigned nblk = blocks_for(std::max<int64_t>(G, 1), tpb);
    int64_t nch = 0, spc = 0;
    if (j->multiband_on) {
        mm_solve_geom sg;
        solve_geometry(j, &sg);  // (checked by stage_compress)
        nch = sg.chunks;
        spc = sg.cols_per_chunk;
    }
    // (each look-back region also holds the K-weighting stage's blocks: sub-tile lanes)
    const unsigned nblk_kw = j->lufs_on ? blocks_for(std::max<int64_t>(G, 1) * (T / std::max(1, j->kweight.tile)),
                                                     LB_THREADS) : 0u;
    RET(setup_control(c, std::max(nblk, nblk_kw), nch, 3 * nch * spc + 3 * nch * spc / 64));  // claim stamps, column-block counts

    EqArgs ea{};
    ea.in = j->in_kind == MM_IN_I16 ? nullptr : static_cast<const float *>(d_in);
    ea.in16 = j->in_kind == MM_IN_I16 ? static_cast<const int16_t *>(d_in) : nullptr;
    ea.N_in = j->frames_in;
    ea.N_proc = N;
    ea.G = G;
    ea.T = T;
    ea.sat.keep = j->sat_keep;
    ea.sat.mix = j->sat_mix;
    ea.sat.drive = j->sat_drive;
    ea.sat.on = j->sat_on;
    ea.sat.tab = nullptr;
    ea.sat.corr = nullptr;
    if (j->sat_on && j->sat_table) {  // the exciter's int16-grid table, uploaded when its key changes
        float *tab;
        uint32_t *corr;
        RET(get_buf(c, "sat_tab", 65536, &tab));
        RET(get_buf(c, "sat_corr", SAT_CORR_WORDS, &corr));
        ea.sat.tab = tab;
        if (j->sat_key == 0 || c->sat_key != j->sat_key) {  // once per table: build the codes, count exceptions
            unsigned *exc;
            RET(get_buf(c, "sat_exc", 1, &exc));
            HIPCHK(c, hipMemcpyAsync(tab, j->sat_table, 65536 * sizeof(float), hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipMemsetAsync(exc, 0, sizeof(unsigned), c->stream));
            RET(launch(c, "sat_corr", sat_corr_kernel, dim3((SAT_CORR_WORDS + 255) / 256), dim3(256), 0, ea.sat, corr,
                       exc));
            unsigned e1 = 1;
            HIPCHK(c, hipMemcpyAsync(&e1, exc, sizeof(unsigned), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            c->sat_codes = e1 == 0;
            c->sat_key = j->sat_key;
        }
        // codes when complete (else, and for A/B: a full-table gather per sample)
        if (c->sat_codes && !getenv("MM_SAT_GATHER")) ea.sat.corr = corr;
        if (getenv("MM_SAT_TANHF")) ea.sat.tab = nullptr, ea.sat.corr = nullptr;  // (A/B: round 5's tanhf alone)
        if (ea.sat.tab && !ea.sat.corr && j->eq.nsec > 0 && N > 0) {
            // the EQ kernel takes the exciter only as tanhf + codes: the table case runs
            // as a pointwise pre-pass into a decoded f32 input, and the EQ without it
            const int64_t n = j->frames_in * ch;
            float *pre;
            RET(get_buf(c, "sat_pre", (size_t)std::max<int64_t>(n, 1), &pre));
            if (n > 0)
                RET(launch(c, "sat_pre", sat_pre_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, ea.in, ea.in16, n,
                           ea.sat, pre));
            ea.in = pre;
            ea.in16 = nullptr;
            ea.sat.on = 0;
        }
    }
    ea.width = j->width;
    ea.width_on = j->width_on && ch == 2;
    ea.q_out = reinterpret_cast<int16_t *>(q1);
    if (j->eq.nsec > 0) RET(get_buf(c, "eq_xs", (size_t)TG * 2, &ea.xs));
    if (G > 0) {
        // --- stage A: saturation -> EQ -> width -> int16 (AME:55-63)
        if (j->eq.nsec == 0) {
            const unsigned nf = blocks_for(N, 256);
            if (ch == 2) RET(launch(c, "pre_pointwise", pre_pointwise_kernel<2>, dim3(nf), dim3(256), 0, ea));
            else RET(launch(c, "pre_pointwise", pre_pointwise_kernel<1>, dim3(nf), dim3(256), 0, ea));
        } else {
            fill_sos(ea.sos, j->eq, j->eq.nsec);
            LbArgs lb{};
            RET(upload_tables(c, "eq", j->eq, lb));
            RET(lb_prepare(c, nblk, ch, lb, 0));
            RET(launch_eq(c, j->eq.nsec, ch, nblk, ea, lb, K));
        }
    }
    short2 *mix = q1;
    const unsigned nb = blocks_for(std::max<int64_t>(G, 1), 256);
    if (j->multiband_on && G > 0) {
        // --- stage B: crossover + band quantisation (AME:196-206)
        short2 *bands[3];
        RET(get_buf(c, "band0", TG, &bands[0]));
        RET(get_buf(c, "band1", TG, &bands[1]));
        RET(get_buf(c, "band2", TG, &bands[2]));
        XoArgs xa{};
        xa.N_proc = N;
        xa.G = G;
        xa.T = T;
        fill_sos(xa.sos, j->xover, 4);
        xa.q_in = reinterpret_cast<const int16_t *>(q1);
        for (int b = 0; b < 3; ++b) xa.band[b] = reinterpret_cast<int16_t *>(bands[b]);
        double *tile_e;  // [3][E, tail][G]
        RET(get_buf(c, "comp_tile_e", (size_t)6 * G, &tile_e));
        for (int b = 0; b < 3; ++b) {
            xa.E[b] = tile_e + (size_t)(2 * b) * G;
            xa.tail[b] = tile_e + (size_t)(2 * b + 1) * G;
            const int r = j->band[b].look % T;
            xa.tail_from[b] = r ? T - r : T;
        }
        LbArgs lb{};
        RET(upload_tables(c, "xover", j->xover, lb));
        if ((size_t)T * 8 * sizeof(double) <= (size_t)lb_lds_bytes<8, 1>())  // (the weights alias its LDS)
            RET(upload_zw(c, "xover", j->xover, T, &xa.zw));
        RET(lb_prepare(c, nblk, ch, lb, 1));
        if (ch == 2)
            RET(launch(c, "xover", xover_kernel<2>, dim3(nblk), dim3(LB_THREADS), lb_lds_bytes<8, 2>(), xa, lb,
                       (int64_t)K));
        else
            RET(launch(c, "xover", xover_kernel<1>, dim3(nblk), dim3(LB_THREADS), lb_lds_bytes<8, 1>(), xa, lb,
                       (int64_t)K));

        // --- stage C: 3-band compressor + overlay (AME:207-210)
        short2 *q2;
        RET(stage_compress(c, j, bands, tile_e, &q2));
        mix = q2;
    } else {
        c->comp_on = false;
    }
    c->mix = mix;
    c->staged = true;
    return MM_OK;
}

// ------------------------------------------------------------ K-weighting
// Loudness geometry on the device (segment bounds; per-block segment ranges),
// uploaded only when the job's geometry changes.
static int upload_geometry(mm_ctx *c) {
    const mm_job *j = &c->job;
    std::vector<int64_t> key;
    key.reserve((size_t)(j->n_segs + 3 + 2 * j->n_blocks));
    key.push_back(j->n_segs);
    key.insert(key.end(), j->seg_bounds, j->seg_bounds + j->n_segs + 1);
    key.push_back(j->n_blocks);
    key.insert(key.end(), j->block_lo, j->block_lo + j->n_blocks);
    key.insert(key.end(), j->block_hi, j->block_hi + j->n_blocks);
    RET(get_buf(c, "kw_bounds", (size_t)j->n_segs + 1, &c->seg_bounds_dev));
    RET(get_buf(c, "gate_s0", (size_t)j->n_blocks, &c->blk_s0));
    RET(get_buf(c, "gate_s1", (size_t)j->n_blocks, &c->blk_s1));
    if (key == c->geom_cache) return MM_OK;
    std::vector<int32_t> s0((size_t)j->n_blocks), s1((size_t)j->n_blocks);
    const int64_t *B = j->seg_bounds, S = j->n_segs;
    for (int64_t b = 0; b < j->n_blocks; ++b) {  // as mm_gate_loudness
        s0[b] = (int32_t)std::min<int64_t>(std::lower_bound(B, B + S + 1, j->block_lo[b]) - B, S);
        s1[b] = (int32_t)std::min<int64_t>(std::lower_bound(B, B + S + 1, j->block_hi[b]) - B, S);
    }
    HIPCHK(c, hipMemcpyAsync(c->seg_bounds_dev, j->seg_bounds, (S + 1) * sizeof(int64_t), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(c->blk_s0, s0.data(), s0.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->blk_s1, s1.data(), s1.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // host vectors are transient
    c->geom_cache = key;
    return MM_OK;
}

// ---- numpy's float32 np.sum as a program (gate.hip kw_blocks_kernel) ----------
// The reduction tree of np.sum over n contiguous float32 values: 8192-element
// buffer chunks summed in order, each chunk numpy's pairwise recursion (leaves of
// <= 128 elements).  Serialised as gate.hip's program layout.
struct PwBuild {
    std::vector<int32_t> loff, llen;        // leaves in order
    std::vector<int32_t> na, nb, nh;        // nodes: operands (>= 0 leaf, < 0 node ~k) and height
    std::vector<int32_t> chunk_leaf;
};
static int32_t pw_node(PwBuild &b, int32_t va, int32_t vb, int32_t ha, int32_t hb, int32_t *h) {
    b.na.push_back(va);
    b.nb.push_back(vb);
    *h = std::max(ha, hb) + 1;
    b.nh.push_back(*h);
    return ~(int32_t)(b.na.size() - 1);
}
static int32_t pw_rec(PwBuild &b, int32_t off, int32_t m, int32_t *h) {
    if (m <= 128) {  // numpy: m < 8 sequential, else eight accumulators + tail
        b.loff.push_back(off);
        b.llen.push_back(m);
        *h = 0;
        return (int32_t)b.loff.size() - 1;
    }
    int32_t n2 = m / 2;
    n2 -= n2 % 8;
    int32_t ha, hb;
    const int32_t va = pw_rec(b, off, n2, &ha);
    const int32_t vb = pw_rec(b, off + n2, m - n2, &hb);
    return pw_node(b, va, vb, ha, hb, h);
}
// appends the program of np.sum over n elements to `out`
static void pw_build(int64_t n, std::vector<int32_t> &out) {
    PwBuild b;
    int32_t acc = 0, hacc = 0;
    const int64_t nch = (n + KB_CHUNK - 1) / KB_CHUNK;
    for (int64_t c = 0; c < nch; ++c) {
        b.chunk_leaf.push_back((int32_t)b.loff.size());
        int32_t h;
        const int32_t v = pw_rec(b, (int32_t)(c * KB_CHUNK), (int32_t)std::min<int64_t>(KB_CHUNK, n - c * KB_CHUNK), &h);
        if (c == 0) {  // res = 0 + pairwise(chunk 0): exact (sums of squares are >= +0)
            acc = v;
            hacc = h;
        } else {
            acc = pw_node(b, acc, v, hacc, h, &hacc);
        }
    }
    b.chunk_leaf.push_back((int32_t)b.loff.size());
    const int32_t nl = (int32_t)b.loff.size(), nn = (int32_t)b.na.size();
    // nodes sorted by height (stable): a level reads only lower ones
    std::vector<int32_t> order(nn), pos(nn);
    for (int32_t k = 0; k < nn; ++k) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return b.nh[x] < b.nh[y]; });
    for (int32_t k = 0; k < nn; ++k) pos[order[k]] = k;
    auto vidx = [&](int32_t v) { return v >= 0 ? v : nl + pos[~v]; };
    const int32_t nlev = nn ? b.nh[order[nn - 1]] : 0;
    out.push_back(nl);
    out.push_back(nn);
    out.push_back(nlev);
    out.push_back((int32_t)nch);
    out.push_back(n == 0 ? -1 : vidx(acc));
    out.insert(out.end(), b.chunk_leaf.begin(), b.chunk_leaf.end());
    out.insert(out.end(), b.loff.begin(), b.loff.end());
    out.insert(out.end(), b.llen.begin(), b.llen.end());
    for (int32_t k = 0; k < nn; ++k) out.push_back(vidx(b.na[order[k]]));
    for (int32_t k = 0; k < nn; ++k) out.push_back(vidx(b.nb[order[k]]));
    for (int32_t L = 0, k = 0; L <= nlev; ++L) {  // level L: nodes of height L + 1
        while (k < nn && b.nh[order[k]] <= L) ++k;
        out.push_back(k);
    }
}
// The program evaluated on the host with the device's operation order (CPU check
// against np.sum: mm_np_sum_f32).
static float pw_eval(const int32_t *P, const float *x) {
    const int nl = P[0], nn = P[1], nch = P[3], root = P[4];
    const int32_t *loff = P + 5 + nch + 1, *llen = loff + nl, *na = llen + nl, *nb = na + nn;
    std::vector<float> val((size_t)nl + nn);
    for (int li = 0; li < nl; ++li) {
        const float *e = x + loff[li];
        const int len = llen[li];
        float res;
        if (len < 8) {
            res = e[0];
            for (int i = 1; i < len; ++i) res = res + e[i];
        } else {
            float r[8];
            for (int q = 0; q < 8; ++q) r[q] = e[q];
            int i = 8;
            for (; i < len - (len & 7); i += 8)
                for (int q = 0; q < 8; ++q) r[q] = r[q] + e[i + q];
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
            for (; i < len; ++i) res = res + e[i];
        }
        val[li] = res;
    }
    for (int k = 0; k < nn; ++k) val[nl + k] = val[na[k]] + val[nb[k]];
    return root < 0 ? 0.0f : val[root];
}

// Per-block programs on the device: blocks [lo_b, lo_b + n_b) of the line; one
// program per distinct length (the clamped last blocks of a track differ).
static int kb_upload(mm_ctx *c, const std::vector<int64_t> &lo, const std::vector<int64_t> &n) {
    std::vector<int64_t> key(lo);
    key.insert(key.end(), n.begin(), n.end());
    const size_t nb = lo.size();
    RET(get_buf(c, "kb_lo", std::max<size_t>(nb, 1), &c->kb_lo));
    RET(get_buf(c, "kb_prog_of", std::max<size_t>(nb, 1), &c->kb_prog_of));
    RET(get_buf(c, "kb_n", std::max<size_t>(nb, 1), &c->kb_n));
    if (key == c->kb_cache && c->kb_prog) return MM_OK;
    std::map<int64_t, int32_t> at;
    std::vector<int32_t> prog, of(nb), n32(nb);
    int nvals = 1, pints = 4;
    for (size_t b = 0; b < nb; ++b) {
        if (n[b] < 0 || n[b] > 16 * KB_CHUNK) return set_err(c, MM_ERR_ARG, "loudness block of %lld frames", (long long)n[b]);
        auto it = at.find(n[b]);
        if (it == at.end()) {
            const int32_t o = (int32_t)prog.size();
            pw_build(n[b], prog);
            if (prog[o] + prog[o + 1] > KB_VMAX || (int64_t)prog.size() - o > KB_PMAX)
                return set_err(c, MM_ERR_ARG, "loudness block program too large");
            while (prog.size() % 4) prog.push_back(0);  // (16-byte aligned programs: int4 copies)
            nvals = std::max(nvals, prog[o] + prog[o + 1]);
            pints = std::max(pints, (int)(prog.size() - o));
            it = at.emplace(n[b], o).first;
        }
        of[b] = it->second;
        n32[b] = (int32_t)n[b];
    }
    c->kb_prog = nullptr;  // (get_buf may move it: re-fetched below)
    prog.resize(prog.size() + pints, 0);  // every block copies the largest program's length
    RET(get_buf(c, "kb_prog", prog.size(), &c->kb_prog));
    if (nb) {
        HIPCHK(c, hipMemcpyAsync(c->kb_lo, lo.data(), nb * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->kb_prog_of, of.data(), nb * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->kb_n, n32.data(), nb * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->kb_prog, prog.data(), prog.size() * 4, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));  // host vectors are transient
    c->kb_cache = key;
    c->kb_nvals = nvals;
    c->kb_pints = pints;
    return MM_OK;
}

// K-weighting + per-segment energies of the staged mix (device).  Returns the
// device segment-energy vector; `line_end` receives the state after the last
// frame when requested.
static int kweight_launch(mm_ctx *c, const double *carry_in_host, double *line_end, double **seg_out) {
    const mm_job *j = &c->job;
    const int64_t G = c->G;
    // one lane per sub-tile of kweight.tile frames (design.kweight_sub), `sub` per tile
    const int sub = j->tile / j->kweight.tile;
    const int64_t GS = G * sub;
    double *part, *seg;
    int64_t *part_seg;
    RET(get_buf(c, "kw_part", (size_t)std::max<int64_t>(GS, 1) * 2, &part));
    RET(get_buf(c, "kw_part_seg", (size_t)std::max<int64_t>(GS, 1), &part_seg));
    RET(get_buf(c, "kw_seg", (size_t)j->n_segs, &seg));
    RET(upload_geometry(c));
    LbArgs lb{};
    RET(upload_tables(c, "kweight", j->kweight, lb));
    const unsigned nblk = blocks_for(GS, LB_THREADS);
    RET(lb_prepare(c, nblk, 1, lb, 2));
    if (carry_in_host) {
        double *init;
        RET(get_buf(c, "kw_init", 8, &init));
        HIPCHK(c, hipMemcpyAsync(init, carry_in_host, 4 * sizeof(double), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));  // pageable source
        lb.init = init;
    }
    KwArgs ka{};
    ka.N_proc = j->frames_proc;
    ka.G = GS;
    ka.T = j->kweight.tile;
    ka.Gt = G;
    ka.sub = sub;
    ka.ch = j->channels;
    for (int s_ = 0; s_ < 2; ++s_)
        for (int k = 0; k < 5; ++k) ka.sos[s_][k] = j->kweight.sos[s_][k];
    ka.mix = reinterpret_cast<const int16_t *>(c->mix);
    ka.n_segs = j->n_segs;
    ka.seg_bounds = c->seg_bounds_dev;
    ka.part = part;
    ka.part_seg = part_seg;
    ka.line_end = line_end;
    RET(launch(c, "kweight", kweight_kernel<false>, dim3(nblk), dim3(LB_THREADS), lb_lds_bytes<4, 1>(), ka, lb));
    RET(launch(c, "seg_reduce", seg_reduce_kernel, dim3(blocks_for(j->n_segs, 4)), dim3(256), 0, ka, seg));  // wave per segment
    *seg_out = seg;
    return MM_OK;
}

// The exact loudness of a line (single track or fused timeline, AME:212-218): the
// K-weighting in lfilter's order writing np.square's f32 values, then pyloudnorm's
// block energies in numpy's reduction order (kw_blocks_kernel) into zl [2 nb].
// The block programs must be on the device (kb_upload) before this is queued.
static int kweight_exact(mm_ctx *c, const mm_job &j0, int64_t frames, int n_trk, const int64_t *trk_tile0,
                         const int64_t *trk_end, int64_t nb, double **zl_out) {
    const int64_t G = c->G;
    const int sub = j0.tile / j0.kweight.tile;  // (design.kweight_sub)
    const int64_t GS = G * sub;
    float *sq;
    double *zl;
    const int Tt = j0.tile, TP = (Tt + 3) / 4 * 4;  // padded tile stride (16-byte stores and loads)
    if (((KB_CHUNK - 1) / Tt + 2) * (TP / 4) > KB_LD * KB_THREADS)
        return set_err(c, MM_ERR_ARG, "tile of %d frames: the loudness block loads do not cover a chunk", Tt);
    RET(get_buf(c, "kw_sq", (size_t)(G * TP), &sq));
    RET(get_buf(c, "gate_zl", (size_t)std::max<int64_t>(2 * nb, 2), &zl));
    LbArgs lb{};
    RET(upload_tables(c, "kweight", j0.kweight, lb));
    const unsigned nblk = blocks_for(GS, LB_THREADS);
    RET(lb_prepare(c, nblk, 1, lb, 2));
    KwArgs ka{};
    ka.N_proc = frames;
    ka.G = GS;
    ka.T = j0.kweight.tile;
    ka.Gt = G;
    ka.sub = sub;
    ka.ch = j0.channels;
    for (int s_ = 0; s_ < 2; ++s_)
        for (int k = 0; k < 5; ++k) ka.sos[s_][k] = j0.kweight.sos[s_][k];
    ka.mix = reinterpret_cast<const int16_t *>(c->mix);
    ka.n_trk = n_trk;
    ka.trk_tile0 = trk_tile0;
    ka.trk_end = trk_end;
    ka.sq = sq;
    ka.sq_tp = TP;
    RET(launch(c, "kweight", kweight_kernel<true>, dim3(nblk), dim3(LB_THREADS), lb_lds_bytes<4, 1>(), ka, lb));
    if (nb > 0) {
        KbArgs kb{};
        kb.sq = sq;
        kb.T = Tt;
        kb.TP = TP;
        kb.n_blocks = nb;
        kb.blk_lo = c->kb_lo;
        kb.blk_prog = c->kb_prog_of;
        kb.blk_n = c->kb_n;
        kb.prog = c->kb_prog;
        kb.scale = (float)j0.block_scale;  // Python float * np.float32: the constant rounded to f32 (NEP 50)
        kb.zl = zl;
        kb.stage_floats = ((KB_CHUNK - 1) / Tt + 2) * TP;  // the padded tile runs a chunk can span
        kb.nvals = 2 * c->kb_nvals;  // (two value buffers)
        kb.pints = c->kb_pints;
        const size_t lds = (size_t)kb_lds_bytes(kb.stage_floats, kb.nvals, kb.pints);
        // persistent: as many workgroups as fit at once (a multiple of 8: the XCD-aware block mapping)
        const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(KB_RING == 1 ? 4 : 2, (160 * 1024) / (int64_t)(lds + 64)));  // (and VGPRs)
        const unsigned grid = (unsigned)std::min<int64_t>((nb + 7) / 8 * 8, (int64_t)c->n_cus * per_cu / 8 * 8);
        RET(launch(c, "kw_blocks", kw_blocks_kernel, dim3(std::max(grid, 8u)), dim3(KB_THREADS), lds, kb));
    }
    *zl_out = zl;
    return MM_OK;
}

// Host-returning variant (time-sharded ranks: carry-in state, range end state).
static int kweight_energies(mm_ctx *c, const double *carry_in_host, double *seg_host, double *range_end_host) {
    double *lend, *seg;
    RET(get_buf(c, "kw_lend", 8, &lend));
    RET(kweight_launch(c, carry_in_host, range_end_host ? lend : nullptr, &seg));
    if (range_end_host)
        HIPCHK(c, hipMemcpyAsync(range_end_host, lend, 4 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (seg_host)
        HIPCHK(c, hipMemcpyAsync(seg_host, seg, c->job.n_segs * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    bool conv;
    return chain_check(c, &conv);
}

// the gate: block energies and levels from the segment energies in parallel (unless
// ga.zl already holds them: the exact path), then one workgroup per track
static int gate_launch(mm_ctx *c, GateArgs ga, unsigned n_tracks) {
    if (!ga.zl) {
        RET(get_buf(c, "gate_zl", (size_t)(2 * ga.n_blocks), &ga.zl));
        RET(launch(c, "gate_blocks", gate_blocks_kernel, dim3(blocks_for(ga.n_blocks, GATE_BLK_THREADS)),
                   dim3(GATE_BLK_THREADS), 0, ga));
    }
    return launch(c, "gate", gate_kernel, dim3(n_tracks), dim3(GATE_THREADS), 0, ga);
}

// Whole-track loudness and gain on the device (no host round trip), exactly
// pyloudnorm's block energies.
static int kweight_device(mm_ctx *c) {
    const mm_job *j = &c->job;
    if (getenv("MM_LOUDNESS_SEGMENTS")) {  // (A/B builds: round 5's f64 segment energies)
        double *seg;
        RET(kweight_launch(c, nullptr, nullptr, &seg));
        GateArgs ga{};
        ga.n_blocks = j->n_blocks;
        ga.blk_s0 = c->blk_s0;
        ga.blk_s1 = c->blk_s1;
        ga.seg = seg;
        ga.scale = j->block_scale;
        ga.target = j->lufs_target;
        ga.out = c->gate_out;
        return gate_launch(c, ga, 1);
    }
    {
        std::vector<int64_t> lo(j->block_lo, j->block_lo + j->n_blocks), n((size_t)j->n_blocks);
        for (int64_t b = 0; b < j->n_blocks; ++b) n[b] = j->block_hi[b] - j->block_lo[b];
        RET(kb_upload(c, lo, n));
    }
    double *zl;
    RET(kweight_exact(c, *j, j->frames_proc, 0, nullptr, nullptr, j->n_blocks, &zl));
    // c->gate_out: in the control block's readback area (setup_control)
    GateArgs ga{};
    ga.n_blocks = j->n_blocks;
    ga.target = j->lufs_target;
    ga.out = c->gate_out;
    ga.zl = zl;
    return gate_launch(c, ga, 1);
}

// numpy's float32 np.sum over x[0..n) evaluated on the host through the same
// program the device runs for pyloudnorm's block energies (CPU check of pw_build).
extern "C" int mm_np_sum_f32(const float *x, int64_t n, float *out) {
    if (!out || n < 0 || (n > 0 && !x) || n > 16 * KB_CHUNK) return MM_ERR_ARG;
    std::vector<int32_t> prog;
    pw_build(n, prog);
    *out = pw_eval(prog.data(), x);
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

static int finalize(mm_ctx *c, double gain, const double *gain_dev, int use_gain, void *d_out, bool tail = false) {
    const mm_job *j = &c->job;
    c->tail_readback = false;
    if (c->G == 0) return MM_OK;
    FinArgs fa{};
    fa.N_proc = j->frames_proc;
    fa.G = c->G;
    fa.Gs = c->G;
    fa.g_off = 0;
    fa.T = j->tile;
    fa.ch = j->channels;
    fa.out_kind = j->out_kind;
    fa.use_gain = use_gain;
    fa.gain = gain;
    fa.gain_dev = gain_dev;
    fa.mix = c->mix;
    fa.out = d_out;
    if (tail) RET(attach_tail(c, fa));
    const size_t lds = (size_t)FIN_TILES * (j->tile + 1) * sizeof(short2);
    if (fa.ch == 2)
        return launch(c, "finalize", finalize_kernel<2>, dim3(blocks_for(c->G, FIN_TILES)), dim3(256), lds, fa);
    return launch(c, "finalize", finalize_kernel<1>, dim3(blocks_for(c->G, FIN_TILES)), dim3(256), lds, fa);
}

// The chain is queued without host round trips (enqueue_chain); one sync at the
// end (complete_chain) checks the compressor's convergence (a rare unconverged
// batch is extended and the dependent stages re-run) and reads the loudness.
static int enqueue_tail(mm_ctx *c, const mm_job *j, void *d_out) {
    const bool lufs = j->lufs_on && c->G > 0;
    if (lufs) RET(kweight_device(c));
    RET(finalize(c, 1.0, lufs ? c->gate_out + 1 : nullptr, j->lufs_on, d_out, true));
    return c->tail_readback ? MM_OK : queue_readback(c, lufs);
}

static int enqueue_chain(mm_ctx *c, const mm_job *j, const void *d_in, void *d_out) {
    RET(stage_front(c, j, d_in));
    return enqueue_tail(c, j, d_out);
}

static int complete_chain(mm_ctx *c, const mm_job *j, void *d_out, mm_result *res) {
    RbKeep keep;
    for (;;) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        bool converged;
        RET(evaluate_chain(c, &converged));
        if (converged) break;
        rb_keep(c, keep);
        RET(comp_sweeps(c, 8));
        RET(comp_back(c));
        RET(enqueue_tail(c, j, d_out));
    }
    rb_finish(c, keep);
    if (res) {
        const bool lufs = j->lufs_on && c->G > 0;
        const double *lg = reinterpret_cast<const double *>(c->rb + RB_LG);
        res->loudness = j->lufs_on ? (lufs ? lg[0] : -INFINITY) : NAN;  // no frames: pyloudnorm raised earlier
        res->gain_linear = j->lufs_on ? (lufs ? lg[1] : INFINITY) : 1.0;
        res->frames_out = j->frames_proc;
        res->comp_iters = c->comp_iters;
        res->comp_active = 0;
        const int32_t *tot = reinterpret_cast<const int32_t *>(c->rb + RB_TOTALS);
        for (int64_t k = 0; k < 3 * comp_chunks(c); ++k) res->comp_active += tot[k];
        res->comp_walked = c->comp_on ? (int64_t) * reinterpret_cast<const unsigned long long *>(c->rb + RB_WALKED) : 0;
        res->comp_jumped = c->comp_on ? (int64_t) * reinterpret_cast<const unsigned long long *>(c->rb + RB_WALKED + 8) : 0;
    }
    return MM_OK;
}

static int master_device(mm_ctx *c, const mm_job *j, const void *d_in, void *d_out, mm_result *res) {
    RET(enqueue_chain(c, j, d_in, d_out));
    return complete_chain(c, j, d_out, res);
}

// Stage the chunk chain of a range (time-sharded ranks) to convergence.
static int stage_chunks(mm_ctx *c, const mm_job *j, const void *d_in) {
    RET(stage_front(c, j, d_in));
    for (;;) {
        bool converged;
        RET(chain_check(c, &converged));
        if (converged) return MM_OK;
        RET(comp_sweeps(c, 8));
        RET(comp_back(c));
    }
}

// ------------------------------------------------------------ fused batch
// Tracks with the same settings mastered as ONE timeline (BASELINE C3/C5 on one
// GPU).  Track i occupies whole chunks [off_i, off_i + n_i * CF) of it, its last
// chunk zero-padded; every per-chunk stage (EQ, crossover, compressor: AME:48-77
// restarts them per chunk) then runs once over all tracks with the single-track
// kernels, and the padding changes none of a track's frames because it follows
// them and every stage is causal.  The K-weighting line restarts at each track
// start and gives padding frames zero energy; the gating runs one block per
// track; finalize writes every track to its own output.  One launch per stage
// covers the whole batch (n times one track's lanes), which fills the GPU where a
// single track's latency-bound launches leave most SIMDs idle.
struct FusedPlan {
    std::vector<int64_t> off;  // [n + 1] first timeline frame of each track (and the end)
    std::vector<int64_t> nch;  // [n] chunks of each track
    int64_t P = 0;             // timeline frames
    // loudness geometry on the device
    int64_t n_segs = 0, n_blocks = 0;
    int64_t *bounds = nullptr, *trk_blk = nullptr, *trk_tile0 = nullptr, *trk_end = nullptr;
    int32_t *s0 = nullptr, *s1 = nullptr;
};

static bool same_iir(const mm_iir &a, const mm_iir &b) { return memcmp(&a, &b, sizeof a) == 0; }

// jobs that differ only in their track (length, loudness geometry): one timeline
static bool fusable(const mm_job *J, int n) {
    const mm_job &a = J[0];
    for (int i = 0; i < n; ++i) {
        const mm_job &b = J[i];
        if (b.frames_proc <= 0) return false;
        if (i == 0) continue;
        if (b.channels != a.channels || b.rate != a.rate || b.tile != a.tile || b.tiles_per_chunk != a.tiles_per_chunk ||
            b.sat_keep != a.sat_keep || b.sat_mix != a.sat_mix || b.sat_drive != a.sat_drive || b.sat_on != a.sat_on ||
            (b.sat_table == nullptr) != (a.sat_table == nullptr) || b.sat_key != a.sat_key ||
            b.width != a.width || b.width_on != a.width_on || b.multiband_on != a.multiband_on ||
            b.lufs_on != a.lufs_on || b.out_kind != a.out_kind || b.in_kind != a.in_kind ||
            b.comp_warmup != a.comp_warmup || b.comp_max_iters != a.comp_max_iters || b.comp_super != a.comp_super)
            return false;
        if (!same_iir(a.eq, b.eq)) return false;
        if (a.lufs_on && (b.lufs_target != a.lufs_target || b.block_scale != a.block_scale || !same_iir(a.kweight, b.kweight)))
            return false;
        if (a.multiband_on) {
            if (!same_iir(a.xover, b.xover)) return false;
            for (int k = 0; k < 3; ++k) {
                const mm_band &x = a.band[k], &y = b.band[k];
                if (x.thresh_rms != y.thresh_rms || x.attack_frames != y.attack_frames ||
                    x.release_frames != y.release_frames || x.look != y.look || x.r0 != y.r0)
                    return false;
                const bool keyed = x.lut_key != 0 && y.lut_key != 0;
                if (keyed ? x.lut_key != y.lut_key
                          : (x.lut != y.lut && memcmp(x.lut, y.lut, (size_t)32769 * 4 * sizeof(double)) != 0))
                    return false;
            }
        }
    }
    return true;
}

static bool fused_layout(const mm_job *J, int n, FusedPlan *p) {
    const int64_t CF = (int64_t)J[0].tile * J[0].tiles_per_chunk;
    p->off.assign((size_t)n + 1, 0);
    p->nch.assign((size_t)n, 0);
    for (int i = 0; i < n; ++i) {
        p->nch[i] = (J[i].frames_proc + CF - 1) / CF;
        p->off[i + 1] = p->off[i] + p->nch[i] * CF;
    }
    p->P = p->off[n];
    return p->P < ((int64_t)1 << 31);  // 32-bit frame indexing
}

// Loudness geometry of the timeline, uploaded before anything is queued (its one
// sync then waits on nothing): every track's segment bounds shifted to its
// offset (a bound shared with the previous track's end is not repeated; the gap
// between a track's last bound and the next track start is a padding segment
// no gating block reads), every track's blocks as segment ranges of that list.
static int fused_geometry(mm_ctx *c, const mm_job *J, int n, FusedPlan *p) {
    const int T = J[0].tile;
    std::vector<int64_t> bounds, tblk((size_t)n + 1), tt0((size_t)n), tend((size_t)n);
    std::vector<int32_t> s0, s1;
    for (int i = 0; i < n; ++i) {
        const mm_job &j = J[i];
        const int64_t o = p->off[i];
        int64_t base;
        if (!bounds.empty() && bounds.back() == o + j.seg_bounds[0]) {
            base = (int64_t)bounds.size() - 1;
        } else {
            base = (int64_t)bounds.size();
            bounds.push_back(o + j.seg_bounds[0]);
        }
        for (int64_t s = 1; s <= j.n_segs; ++s) bounds.push_back(o + j.seg_bounds[s]);
        tblk[i] = (int64_t)s0.size();
        const int64_t *B = j.seg_bounds, S = j.n_segs;
        for (int64_t b = 0; b < j.n_blocks; ++b) {  // as mm_gate_loudness
            s0.push_back((int32_t)(base + std::min<int64_t>(std::lower_bound(B, B + S + 1, j.block_lo[b]) - B, S)));
            s1.push_back((int32_t)(base + std::min<int64_t>(std::lower_bound(B, B + S + 1, j.block_hi[b]) - B, S)));
        }
        tt0[i] = o / T;
        tend[i] = o + j.frames_proc;
    }
    tblk[n] = (int64_t)s0.size();
    {  // the exact path's blocks: every track's own blocks at its timeline offset
        std::vector<int64_t> lo, len;
        for (int i = 0; i < n; ++i)
            for (int64_t b = 0; b < J[i].n_blocks; ++b) {
                lo.push_back(p->off[i] + J[i].block_lo[b]);
                len.push_back(J[i].block_hi[b] - J[i].block_lo[b]);
            }
        RET(kb_upload(c, lo, len));
    }
    if (bounds.back() < p->P) bounds.push_back(p->P);  // the last track's padding
    p->n_segs = (int64_t)bounds.size() - 1;
    p->n_blocks = (int64_t)s0.size();
    RET(get_buf(c, "fz_bounds", bounds.size(), &p->bounds));
    RET(get_buf(c, "fz_trk_blk", tblk.size(), &p->trk_blk));
    RET(get_buf(c, "fz_trk_tile0", tt0.size(), &p->trk_tile0));
    RET(get_buf(c, "fz_trk_end", tend.size(), &p->trk_end));
    RET(get_buf(c, "fz_s0", std::max<size_t>(s0.size(), 1), &p->s0));
    RET(get_buf(c, "fz_s1", std::max<size_t>(s1.size(), 1), &p->s1));
    HIPCHK(c, hipMemcpyAsync(p->bounds, bounds.data(), bounds.size() * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(p->trk_blk, tblk.data(), tblk.size() * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(p->trk_tile0, tt0.data(), tt0.size() * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(p->trk_end, tend.data(), tend.size() * 8, hipMemcpyHostToDevice, c->stream));
    if (!s0.empty()) {
        HIPCHK(c, hipMemcpyAsync(p->s0, s0.data(), s0.size() * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(p->s1, s1.data(), s1.size() * 4, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));  // host vectors are transient
    return MM_OK;
}

// K-weighting (a line per track), segment energies and per-track gating into
// lg[2i] = L, lg[2i+1] = gain.
static int fused_loudness(mm_ctx *c, const mm_job &j0, int n, const FusedPlan &p, double *lg) {
    if (!getenv("MM_LOUDNESS_SEGMENTS")) {  // exact block energies (the programs: fused_geometry)
        double *zl;
        RET(kweight_exact(c, j0, p.P, n, p.trk_tile0, p.trk_end, p.n_blocks, &zl));
        GateArgs ga{};
        ga.n_blocks = p.n_blocks;
        ga.target = j0.lufs_target;
        ga.out = lg;
        ga.trk_blk = p.trk_blk;
        ga.zl = zl;
        return gate_launch(c, ga, (unsigned)n);
    }
    const int64_t G = c->G;
    const int sub = j0.tile / j0.kweight.tile;  // (design.kweight_sub)
    const int64_t GS = G * sub;
    double *part, *seg;
    int64_t *part_seg;
    RET(get_buf(c, "kw_part", (size_t)GS * 2, &part));
    RET(get_buf(c, "kw_part_seg", (size_t)GS, &part_seg));
    RET(get_buf(c, "kw_seg", (size_t)p.n_segs, &seg));
    LbArgs lb{};
    RET(upload_tables(c, "kweight", j0.kweight, lb));
    const unsigned nblk = blocks_for(GS, LB_THREADS);
    RET(lb_prepare(c, nblk, 1, lb, 2));
    KwArgs ka{};
    ka.N_proc = p.P;
    ka.G = GS;
    ka.T = j0.kweight.tile;
    ka.Gt = G;
    ka.sub = sub;
    ka.ch = j0.channels;
    for (int s_ = 0; s_ < 2; ++s_)
        for (int k = 0; k < 5; ++k) ka.sos[s_][k] = j0.kweight.sos[s_][k];
    ka.mix = reinterpret_cast<const int16_t *>(c->mix);
    ka.n_segs = p.n_segs;
    ka.seg_bounds = p.bounds;
    ka.part = part;
    ka.part_seg = part_seg;
    ka.n_trk = n;
    ka.trk_tile0 = p.trk_tile0;
    ka.trk_end = p.trk_end;
    RET(launch(c, "kweight", kweight_kernel<false>, dim3(nblk), dim3(LB_THREADS), lb_lds_bytes<4, 1>(), ka, lb));
    RET(launch(c, "seg_reduce", seg_reduce_kernel, dim3(blocks_for(p.n_segs, 4)), dim3(256), 0, ka, seg));
    GateArgs ga{};
    ga.n_blocks = p.n_blocks;
    ga.blk_s0 = p.s0;
    ga.blk_s1 = p.s1;
    ga.seg = seg;
    ga.scale = j0.block_scale;
    ga.target = j0.lufs_target;
    ga.out = lg;
    ga.trk_blk = p.trk_blk;
    return gate_launch(c, ga, (unsigned)n);
}

static int fused_finalize(mm_ctx *c, const mm_job *J, int n, const FusedPlan &p, const double *lg, void *const *d_out) {
    const mm_job &j0 = J[0];
    const int T = j0.tile;
    const size_t lds = (size_t)FIN_TILES * (T + 1) * sizeof(short2);
    c->tail_readback = false;
    for (int i = 0; i < n; ++i) {
        FinArgs fa{};
        fa.N_proc = J[i].frames_proc;
        fa.G = p.nch[i] * j0.tiles_per_chunk;
        fa.Gs = c->G;
        fa.g_off = p.off[i] / T;
        fa.T = T;
        fa.ch = j0.channels;
        fa.out_kind = j0.out_kind;
        fa.use_gain = j0.lufs_on;
        fa.gain = 1.0;
        fa.gain_dev = j0.lufs_on ? lg + 2 * i + 1 : nullptr;
        fa.mix = c->mix;
        fa.out = d_out[i];
        if (i == n - 1 && fa.G > 0) RET(attach_tail(c, fa));
        const dim3 grid(blocks_for(fa.G, FIN_TILES));
        if (fa.ch == 2) RET(launch(c, "finalize", finalize_kernel<2>, grid, dim3(256), lds, fa));
        else RET(launch(c, "finalize", finalize_kernel<1>, grid, dim3(256), lds, fa));
    }
    return MM_OK;
}

// Queue a fused unit: loudness geometry (uploaded first: its sync waits on an
// idle stream), the input timeline (in place when the tracks already lie back to
// back on whole chunks, else gathered with the padding zeroed), the chunk stages,
// loudness and the per-track finalize.
static int fused_enqueue(mm_ctx *c, int n, const mm_job *J, const void *const *d_in, void *const *d_out, FusedPlan &p) {
    const mm_job &j0 = J[0];
    const bool lufs = j0.lufs_on != 0;
    if (lufs) RET(fused_geometry(c, J, n, &p));
    const size_t fb = (size_t)j0.channels * (j0.in_kind == MM_IN_I16 ? 2 : 4);
    bool in_place = true;
    for (int i = 0; i < n && in_place; ++i)
        in_place = J[i].frames_in == p.off[i + 1] - p.off[i] &&
                   static_cast<const char *>(d_in[i]) == static_cast<const char *>(d_in[0]) + p.off[i] * fb;
    const void *tin = d_in[0];
    if (!in_place) {
        char *buf;
        RET(get_buf(c, "fz_in", (size_t)p.P * fb, &buf));
        for (int i = 0; i < n; ++i) {
            const int64_t len = p.off[i + 1] - p.off[i], nin = std::min(J[i].frames_in, len);
            if (nin > 0)
                HIPCHK(c, hipMemcpyAsync(buf + p.off[i] * fb, d_in[i], nin * fb, hipMemcpyDeviceToDevice, c->stream));
            if (len > nin) HIPCHK(c, hipMemsetAsync(buf + (p.off[i] + nin) * fb, 0, (len - nin) * fb, c->stream));
        }
        tin = buf;
    }
    mm_job tj = j0;  // the timeline as one job (loudness is per track)
    tj.frames_in = tj.frames_proc = p.P;
    tj.lufs_on = 0;
    RET(stage_front(c, &tj, tin));
    double *lg;
    RET(get_buf(c, "fz_lg", (size_t)2 * n, &lg));
    if (lufs) RET(fused_loudness(c, j0, n, p, lg));
    RET(fused_finalize(c, J, n, p, lg, d_out));
    return c->tail_readback ? MM_OK : queue_readback(c, lufs);
}

static int fused_complete(mm_ctx *c, int n, const mm_job *J, void *const *d_out, mm_result *res, const FusedPlan &p) {
    const mm_job &j0 = J[0];
    const bool lufs = j0.lufs_on != 0;
    double *lg;
    RET(get_buf(c, "fz_lg", (size_t)2 * n, &lg));
    RbKeep keep;
    for (;;) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        bool converged;
        RET(evaluate_chain(c, &converged));
        if (converged) break;
        rb_keep(c, keep);
        RET(comp_sweeps(c, 8));
        RET(comp_back(c));
        if (lufs) RET(fused_loudness(c, j0, n, p, lg));
        RET(fused_finalize(c, J, n, p, lg, d_out));
        if (!c->tail_readback) RET(queue_readback(c, lufs));
    }
    rb_finish(c, keep);
    if (!res) return MM_OK;
    std::vector<double> l2((size_t)2 * n, 0.0);
    if (lufs) HIPCHK(c, hipMemcpy(l2.data(), lg, l2.size() * sizeof(double), hipMemcpyDeviceToHost));
    const int64_t nchk = comp_chunks(c), CF = (int64_t)j0.tile * j0.tiles_per_chunk;
    const int32_t *tot = reinterpret_cast<const int32_t *>(c->rb + RB_TOTALS);
    const int64_t walked = c->comp_on ? (int64_t) * reinterpret_cast<const unsigned long long *>(c->rb + RB_WALKED) : 0;
    const int64_t jumped = c->comp_on ? (int64_t) * reinterpret_cast<const unsigned long long *>(c->rb + RB_WALKED + 8) : 0;
    for (int i = 0; i < n; ++i) {
        mm_result &r = res[i];
        r.loudness = lufs ? l2[2 * i] : NAN;
        r.gain_linear = lufs ? l2[2 * i + 1] : 1.0;
        r.frames_out = J[i].frames_proc;
        r.comp_iters = c->comp_iters;  // one solve for the whole unit
        r.comp_active = 0;
        for (int b = 0; b < 3 && c->comp_on; ++b)
            for (int64_t k = p.off[i] / CF; k < p.off[i + 1] / CF; ++k) r.comp_active += tot[b * nchk + k];
        // the unit's solve statistics are reported once, on its first track (sums over
        // a batch's results then count every unit once)
        r.comp_walked = i == 0 ? walked : 0;
        r.comp_jumped = i == 0 ? jumped : 0;
    }
    return MM_OK;
}

// A unit of a batch: one track, or consecutive same-settings tracks fused into one
// timeline.  A run of such tracks is split into max(2, ceil(frames / cap)) units of
// about equal length (cap MM_FUSE_MAX_FRAMES, default 150 M frames): two units in
// flight on two streams overlap one unit's latency-bound tail with the other's
// front (C3 8 x 3 min: 14.5 G frames/s as 2 units, 14.2 as 1, 13.7 as 4; C5 16 x 3
// min at 96 kHz: 12.6 as 2, 12.3 as 4, 12.0 as 1, 11.0 unfused), and the cap
// keeps a unit's compacted envelope arrays to a few GB.
struct BatchUnit {
    int first = 0, count = 1;
    FusedPlan plan;
};

static std::vector<BatchUnit> batch_units(const mm_job *J, int n) {
    int64_t cap = 150000000;
    if (const char *e = getenv("MM_FUSE_MAX_FRAMES")) cap = std::max<int64_t>(1, atoll(e));
    const bool fuse = !getenv("MM_BATCH_STREAMS_ONLY");
    auto padded = [&](int i) {
        const int64_t CF = (int64_t)J[i].tile * J[i].tiles_per_chunk;
        return (J[i].frames_proc + CF - 1) / CF * CF;
    };
    std::vector<BatchUnit> units;
    for (int i = 0; i < n;) {
        int run = 1;  // maximal run of tracks fusable with track i
        int64_t total = padded(i);
        while (fuse && i + run < n) {
            const mm_job pair[2] = {J[i], J[i + run]};
            if (!fusable(pair, 2)) break;
            total += padded(i + run);
            ++run;
        }
        const int parts = (int)std::min<int64_t>(run, std::max<int64_t>(std::min(2, run), (total + cap - 1) / cap));
        int64_t acc = 0;
        int k = i;
        for (int q = 0; q < parts; ++q) {  // close unit q once it holds about (q+1)/parts of the run
            BatchUnit u;
            u.first = k;
            if (q + 1 == parts) {
                k = i + run;
            } else {
                const int64_t goal = total * (q + 1) / parts;
                acc += padded(k++);
                while (k < i + run - (parts - q - 1) && acc + padded(k) / 2 <= goal) acc += padded(k++);
            }
            u.count = k - u.first;
            if (u.count > 1 && !fused_layout(J + u.first, u.count, &u.plan)) {  // over 2^31 frames: one by one
                for (int t = u.first; t < k; ++t) {
                    BatchUnit v;
                    v.first = t;
                    units.push_back(std::move(v));
                }
                continue;
            }
            units.push_back(std::move(u));
        }
        i += run;
    }
    return units;
}

// =================================================================== C-ABI
extern "C" {

int mm_version(void) { return MM_ABI_VERSION; }

int mm_solve_geometry(const mm_job *j, mm_solve_geom *out) {
    if (!j || !out) return MM_ERR_ARG;
    return solve_geometry(j, out);
}

#ifndef MM_SOURCE_SHA
#define MM_SOURCE_SHA "unknown"
#endif
const char *mm_source_sha(void) { return MM_SOURCE_SHA; }

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
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
        c->n_cus = ncu;
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
    for (int b = 0; b < 2; ++b) {
        if (c->pin[b]) hipHostFree(c->pin[b]);
        if (c->pin_ev[b]) hipEventDestroy(c->pin_ev[b]);
    }
    if (c->rb) hipHostFree(c->rb);
    for (mm_ctx *k : c->children) mm_destroy(k);
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

int mm_master_device(mm_ctx *c, const mm_job *j, const void *d_in, void *d_out, mm_result *res) {
    if (!c) return MM_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    return master_device(c, j, d_in, d_out, res);
}

// A batch of independent tracks (BASELINE C3/C5 on one GPU), cut into units
// (batch_units: same-settings runs fused into one timeline, else single tracks);
// unit u runs on child context u % S (own stream and buffers, S = min(units,
// MM_BATCH_STREAMS)), so up to S units are in flight at once and their
// latency-bound kernels fill each other's idle SIMDs.  Units are completed in
// submission order; a child's next unit is queued as soon as its previous one
// has been checked.
int mm_master_batch(mm_ctx *c, int n, const mm_job *jobs, const void *const *d_in, void *const *d_out,
                    mm_result *res) {
    if (!c || n < 0 || (n > 0 && (!jobs || !d_in || !d_out))) return set_err(c, MM_ERR_ARG, "bad arguments");
    HIPCHK(c, hipSetDevice(c->device));
    for (int i = 0; i < n; ++i) RET(validate(c, &jobs[i]));
    std::vector<BatchUnit> units = batch_units(jobs, n);
    const int nu = (int)units.size();
    const int S = std::min(nu, MM_BATCH_STREAMS);
    while ((int)c->children.size() < S) {
        mm_ctx *k = nullptr;
        if (mm_create(c->device, &k) != MM_OK) return set_err(c, MM_ERR_HIP, "cannot create a batch stream");
        c->children.push_back(k);
    }
    for (int s = 0; s < S; ++s) {
        c->children[s]->timing = c->timing;
    }
    auto enqueue = [&](mm_ctx *k, BatchUnit &u) {
        const int f = u.first;
        if (u.count == 1) return enqueue_chain(k, &jobs[f], d_in[f], d_out[f]);
        return fused_enqueue(k, u.count, jobs + f, d_in + f, d_out + f, u.plan);
    };
    auto complete = [&](mm_ctx *k, BatchUnit &u) {
        const int f = u.first;
        if (u.count == 1) return complete_chain(k, &jobs[f], d_out[f], res ? &res[f] : nullptr);
        return fused_complete(k, u.count, jobs + f, d_out + f, res ? res + f : nullptr, u.plan);
    };
    std::vector<int> cur((size_t)S, -1);
    int next = 0;
    auto fail = [&](mm_ctx *k) {
        set_err(c, MM_ERR_STATE, "batch job: %s", k->err);
        for (int s = 0; s < S; ++s) hipStreamSynchronize(c->children[s]->stream);
        return MM_ERR_STATE;
    };
    for (int s = 0; s < S && next < nu; ++s, ++next) {
        cur[s] = next;
        if (enqueue(c->children[s], units[next]) != MM_OK) return fail(c->children[s]);
    }
    for (int done = 0; done < nu;) {
        for (int s = 0; s < S; ++s) {
            if (cur[s] < 0) continue;
            mm_ctx *k = c->children[s];
            if (complete(k, units[cur[s]]) != MM_OK) return fail(k);
            ++done;
            cur[s] = -1;
            if (next < nu) {
                cur[s] = next;
                if (enqueue(k, units[next]) != MM_OK) return fail(k);
                ++next;
            }
        }
    }
    for (int s = 0; s < S; ++s) {  // per-kernel timing of the children lands in the parent's stats
        mm_ctx *k = c->children[s];
        resolve_events(k);
        for (auto &nm : k->stat_order) {
            auto it = c->stats.find(nm);
            if (it == c->stats.end()) {
                c->stat_order.push_back(nm);
                it = c->stats.emplace(nm, KStat{}).first;
            }
            it->second.ms += k->stats[nm].ms;
            it->second.n += k->stats[nm].n;
        }
        k->stats.clear();
        k->stat_order.clear();
    }
    return MM_OK;
}

int mm_master(mm_ctx *c, const mm_job *j, const void *in, void *out, mm_result *res) {
    if (!c) return MM_ERR_ARG;
    RET(validate(c, j));
    HIPCHK(c, hipSetDevice(c->device));
    char *d_in;
    void *d_out;
    const size_t in_bytes = (size_t)j->frames_in * j->channels * (j->in_kind == MM_IN_I16 ? 2 : 4);
    const size_t out_bytes = (size_t)j->frames_proc * j->channels * (j->out_kind == MM_OUT_I16 ? 2 : 4);
    RET(get_buf(c, "host_in", std::max<size_t>(in_bytes, 1), &d_in));
    char *ob;
    RET(get_buf(c, "host_out", std::max<size_t>(out_bytes, 1), &ob));
    d_out = ob;
    if (in_bytes) HIPCHK(c, hipMemcpyAsync(d_in, in, in_bytes, hipMemcpyHostToDevice, c->stream));
    RET(master_device(c, j, d_in, d_out, res));
    if (out_bytes) HIPCHK(c, hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    return MM_OK;
}

// ------------------------------------------------------------ WAV files
// RIFF/WAVE codec of the file path (replaces pydub/ffmpeg decode, AME:43, and the
// stdlib `wave` export, AME:98), mirroring mastering_amd/wavio.py: PCM16 or
// IEEE float32 (WAVE_FORMAT_EXTENSIBLE resolved through its subformat), the
// last fmt/data chunk wins, a data chunk running past the end of the file is
// truncated to whole frames.
static uint32_t le32(const unsigned char *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }
static uint16_t le16(const unsigned char *p) { return (uint16_t)(p[0] | p[1] << 8); }

static int wav_parse(mm_ctx *c, FILE *f, const char *path, mm_wav_info *info) {
    unsigned char h[40];
    if (fseeko(f, 0, SEEK_END) != 0) return set_err(c, MM_ERR_ARG, "%s: cannot seek", path);
    const int64_t fsize = (int64_t)ftello(f);
    if (fseeko(f, 0, SEEK_SET) != 0 || fread(h, 1, 12, f) != 12 || memcmp(h, "RIFF", 4) || memcmp(h + 8, "WAVE", 4))
        return set_err(c, MM_ERR_ARG, "%s: not a RIFF/WAVE file", path);
    int64_t pos = 12, data_off = -1, data_size = 0;
    int tag = -1, ch = 0, rate = 0, bits = 0;
    while (pos + 8 <= fsize) {
        if (fseeko(f, pos, SEEK_SET) != 0 || fread(h, 1, 8, f) != 8) break;
        const int64_t size = le32(h + 4);
        if (!memcmp(h, "fmt ", 4)) {
            const size_t nb = (size_t)std::min<int64_t>(std::min<int64_t>(size, 40), fsize - pos - 8);
            unsigned char b[40] = {0};
            if (nb < 16 || fread(b, 1, nb, f) != nb) return set_err(c, MM_ERR_ARG, "%s: short fmt chunk", path);
            tag = le16(b);
            ch = le16(b + 2);
            rate = (int)le32(b + 4);
            bits = le16(b + 14);
            if (tag == 0xFFFE && nb >= 26) tag = le16(b + 24);
        } else if (!memcmp(h, "data", 4)) {
            data_off = pos + 8;
            data_size = std::min<int64_t>(size, fsize - data_off);
        }
        pos += 8 + size + (size & 1);
    }
    if (tag < 0 || data_off < 0) return set_err(c, MM_ERR_ARG, "%s: missing fmt or data chunk", path);
    if (!((tag == 1 && bits == 16) || (tag == 3 && bits == 32)))
        return set_err(c, MM_ERR_ARG, "%s: unsupported WAV format tag=%d bits=%d", path, tag, bits);
    if (ch < 1 || rate < 1) return set_err(c, MM_ERR_ARG, "%s: bad fmt chunk (channels %d, rate %d)", path, ch, rate);
    info->frames = data_size / (ch * bits / 8);
    info->data_offset = data_off;
    info->rate = rate;
    info->channels = ch;
    info->format = tag;
    info->bits = bits;
    return MM_OK;
}

int mm_wav_probe(mm_ctx *c, const char *path, mm_wav_info *info) {
    if (!path || !info) return set_err(c, MM_ERR_ARG, "null argument");
    FILE *f = fopen(path, "rb");
    if (!f) return set_err(c, MM_ERR_ARG, "%s: cannot open", path);
    const int rc = wav_parse(c, f, path, info);
    fclose(f);
    return rc;
}

constexpr size_t PIN_CHUNK = (size_t)8 << 20;  // bytes per staging buffer

static int ensure_pinned(mm_ctx *c) {
    for (int b = 0; b < 2; ++b) {
        if (!c->pin[b]) HIPCHK(c, hipHostMalloc((void **)&c->pin[b], PIN_CHUNK, hipHostMallocDefault));
        if (!c->pin_ev[b]) HIPCHK(c, hipEventCreateWithFlags(&c->pin_ev[b], hipEventDisableTiming));
    }
    return MM_OK;
}

namespace {
struct FileCloser {
    FILE *f;
    ~FileCloser() {
        if (f) fclose(f);
    }
};
}  // namespace

int mm_master_wav(mm_ctx *c, const mm_job *jin, const char *in_path, const char *out_path, mm_result *res) {
    if (!c) return MM_ERR_ARG;
    if (!jin || !in_path || !out_path) return set_err(c, MM_ERR_ARG, "null argument");
    HIPCHK(c, hipSetDevice(c->device));
    FileCloser in{fopen(in_path, "rb")};
    if (!in.f) return set_err(c, MM_ERR_ARG, "%s: cannot open", in_path);
    mm_wav_info wi;
    RET(wav_parse(c, in.f, in_path, &wi));
    mm_job j = *jin;
    j.in_kind = wi.format == 1 ? MM_IN_I16 : MM_IN_F32;
    if (j.frames_in != wi.frames || j.channels != wi.channels || j.rate != wi.rate)
        return set_err(c, MM_ERR_ARG, "%s: job built for %lld frames x %d ch @ %d Hz, file has %lld x %d @ %d", in_path,
                       (long long)j.frames_in, j.channels, j.rate, (long long)wi.frames, wi.channels, wi.rate);
    RET(validate(c, &j));
    const size_t in_bytes = (size_t)wi.frames * wi.channels * (wi.bits / 8);
    const size_t out_bytes = (size_t)j.frames_proc * j.channels * (j.out_kind == MM_OUT_I16 ? 2 : 4);
    if (out_bytes > 0xFFFFFFFFull - 36) return set_err(c, MM_ERR_ARG, "output larger than a RIFF file can hold");
    char *d_in, *d_out;
    RET(get_buf(c, "host_in", std::max<size_t>(in_bytes, 1), &d_in));
    RET(get_buf(c, "host_out", std::max<size_t>(out_bytes, 1), &d_out));
    RET(ensure_pinned(c));
    // file -> pinned -> HBM: chunk k is read while chunk k-1 is in flight
    if (fseeko(in.f, wi.data_offset, SEEK_SET) != 0) return set_err(c, MM_ERR_ARG, "%s: cannot seek", in_path);
    size_t k = 0;
    for (size_t off = 0; off < in_bytes; ++k) {
        const int b = (int)(k & 1);
        const size_t n = std::min(PIN_CHUNK, in_bytes - off);
        if (k >= 2) HIPCHK(c, hipEventSynchronize(c->pin_ev[b]));
        if (fread(c->pin[b], 1, n, in.f) != n) return set_err(c, MM_ERR_ARG, "%s: short read", in_path);
        HIPCHK(c, hipMemcpyAsync(d_in + off, c->pin[b], n, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipEventRecord(c->pin_ev[b], c->stream));
        off += n;
    }
    RET(master_device(c, &j, d_in, d_out, res));
    // HBM -> pinned -> file: chunk k is written while chunk k+1 is copied back
    FileCloser out{fopen(out_path, "wb")};
    if (!out.f) return set_err(c, MM_ERR_ARG, "%s: cannot create", out_path);
    const int tag = j.out_kind == MM_OUT_I16 ? 1 : 3, bits = j.out_kind == MM_OUT_I16 ? 16 : 32;
    const int ba = j.channels * bits / 8;
    unsigned char hdr[44];
    auto put32 = [&](int at, uint32_t v) {
        for (int i = 0; i < 4; ++i) hdr[at + i] = (unsigned char)(v >> (8 * i));
    };
    auto put16 = [&](int at, uint32_t v) {
        hdr[at] = (unsigned char)v;
        hdr[at + 1] = (unsigned char)(v >> 8);
    };
    memcpy(hdr, "RIFF", 4);
    put32(4, (uint32_t)(36 + out_bytes));
    memcpy(hdr + 8, "WAVEfmt ", 8);
    put32(16, 16);
    put16(20, tag);
    put16(22, j.channels);
    put32(24, j.rate);
    put32(28, (uint32_t)j.rate * ba);
    put16(32, ba);
    put16(34, bits);
    memcpy(hdr + 36, "data", 4);
    put32(40, (uint32_t)out_bytes);
    if (fwrite(hdr, 1, 44, out.f) != 44) return set_err(c, MM_ERR_ARG, "%s: write failed", out_path);
    size_t prev_n = 0;
    k = 0;
    for (size_t off = 0; off < out_bytes; ++k) {
        const int b = (int)(k & 1);
        const size_t n = std::min(PIN_CHUNK, out_bytes - off);
        HIPCHK(c, hipMemcpyAsync(c->pin[b], d_out + off, n, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipEventRecord(c->pin_ev[b], c->stream));
        if (k >= 1) {
            HIPCHK(c, hipEventSynchronize(c->pin_ev[b ^ 1]));
            if (fwrite(c->pin[b ^ 1], 1, prev_n, out.f) != prev_n) return set_err(c, MM_ERR_ARG, "%s: write failed", out_path);
        }
        prev_n = n;
        off += n;
    }
    if (k >= 1) {
        const int b = (int)((k - 1) & 1);
        HIPCHK(c, hipEventSynchronize(c->pin_ev[b]));
        if (fwrite(c->pin[b], 1, prev_n, out.f) != prev_n) return set_err(c, MM_ERR_ARG, "%s: write failed", out_path);
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    return MM_OK;
}

int mm_stage_chunks(mm_ctx *c, const mm_job *j, const void *d_in) {
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

// Time-sharded loudness without a host round trip for the energies (VERDICT r03
// item 7): this rank's per-segment K-weighted energies go straight into a zeroed
// device vector of the whole track's segments at seg_offset (a rank's segments are
// consecutive global segments), ONE RCCL sum all-reduce runs in place on the
// context's stream (when a communicator is set up), the whole track's gating runs
// on the device (gate_kernel over the given block -> segment ranges), and finalize
// reads the gain from device memory.  One host synchronisation before (the
// envelope solve's convergence check, as mm_hop_energies) and one after (L).
// Time-sharded loudness with the energy vector in HBM, in three steps a caller can
// compose with any collective between them (the library's communicator, or
// torch.distributed over the same device buffer):
//  1. mm_shard_energies_device: zero the caller's whole-track vector d_full and write
//     this rank's segment energies at seg_offset (a rank's segments are consecutive
//     global ones);
//  2. a sum all-reduce of d_full over the ranks (mm_allreduce_sum_f64_device);
//  3. mm_gate_finalize_device: pyloudnorm's gating of the whole track on the device,
//     the gain towards `target` applied by finalize straight from device memory;
//     returns L and the gain it applied.
int mm_shard_energies_device(mm_ctx *c, const double *carry_in_host, int64_t n_global_segs, int64_t seg_offset,
                             double *d_full) {
    if (!c || !c->staged) return set_err(c, MM_ERR_STATE, "no staged job");
    const int64_t nl = c->job.n_segs;
    if (!d_full || n_global_segs < 1 || seg_offset < 0 || seg_offset + nl > n_global_segs)
        return set_err(c, MM_ERR_ARG, "shard energies: segments [%lld, %lld) outside [0, %lld)",
                       (long long)seg_offset, (long long)(seg_offset + nl), (long long)n_global_segs);
    HIPCHK(c, hipMemsetAsync(d_full, 0, (size_t)n_global_segs * sizeof(double), c->stream));
    if (c->G > 0 && nl > 0) {
        double *seg;
        RET(kweight_launch(c, carry_in_host, nullptr, &seg));
        HIPCHK(c, hipMemcpyAsync(d_full + seg_offset, seg, (size_t)nl * sizeof(double), hipMemcpyDeviceToDevice,
                                 c->stream));
    }
    bool conv;
    RET(chain_check(c, &conv));  // (synchronises the stream: d_full is complete on return)
    return MM_OK;
}

int mm_gate_finalize_device(mm_ctx *c, const double *d_full, int64_t n_global_segs, int64_t n_blocks,
                            const int32_t *blk_s0_host, const int32_t *blk_s1_host, double block_scale,
                            double target, void *d_out, double *loudness_gain_host) {
    if (!c || !c->staged) return set_err(c, MM_ERR_STATE, "no staged job");
    if (!d_full || n_global_segs < 1 || n_blocks < 1 || !blk_s0_host || !blk_s1_host || !loudness_gain_host)
        return set_err(c, MM_ERR_ARG, "gate: bad segment or block geometry");
    for (int64_t b = 0; b < n_blocks; ++b)
        if (blk_s0_host[b] < 0 || blk_s1_host[b] < blk_s0_host[b] || blk_s1_host[b] > n_global_segs)
            return set_err(c, MM_ERR_ARG, "gate: block %lld has segments [%d, %d) outside [0, %lld)",
                           (long long)b, blk_s0_host[b], blk_s1_host[b], (long long)n_global_segs);
    double *gout;
    int32_t *s0, *s1;
    RET(get_buf(c, "shard_gate", 2, &gout));
    RET(get_buf(c, "shard_blk0", (size_t)n_blocks, &s0));
    RET(get_buf(c, "shard_blk1", (size_t)n_blocks, &s1));
    HIPCHK(c, hipMemcpyAsync(s0, blk_s0_host, (size_t)n_blocks * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(s1, blk_s1_host, (size_t)n_blocks * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    GateArgs ga{};
    ga.n_blocks = n_blocks;
    ga.blk_s0 = s0;
    ga.blk_s1 = s1;
    ga.seg = d_full;
    ga.scale = block_scale;
    ga.target = target;
    ga.out = gout;
    RET(gate_launch(c, ga, 1));
    RET(finalize(c, 1.0, gout + 1, 1, d_out));
    // L and the gain finalize applied (gate.hip's device expression, not a host recomputation)
    HIPCHK(c, hipMemcpyAsync(loudness_gain_host, gout, 2 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MM_OK;
}

// Steps 1-3 with the library's own communicator.  `world` is the plan's rank count:
// a multi-rank plan needs this context's RCCL communicator over exactly that many
// ranks, or every rank would gate only its own part of the vector (and return a
// different, wrong loudness) — refused instead.
int mm_shard_loudness_device(mm_ctx *c, const double *carry_in_host, int64_t n_global_segs, int64_t seg_offset,
                             int64_t n_blocks, const int32_t *blk_s0_host, const int32_t *blk_s1_host,
                             double block_scale, double target, int32_t world, void *d_out,
                             double *loudness_gain_host) {
    if (!c) return MM_ERR_ARG;
    if (world < 1) return set_err(c, MM_ERR_ARG, "shard loudness: world %d", world);
    if (world > 1 && (!c->comm || c->nranks != world))
        return set_err(c, MM_ERR_STATE, "shard loudness: a %d-rank plan needs this context's communicator over %d "
                       "ranks (have %d)", world, world, c->comm ? c->nranks : 0);
    double *full;
    RET(get_buf(c, "shard_seg", (size_t)std::max<int64_t>(n_global_segs, 1), &full));
    RET(mm_shard_energies_device(c, carry_in_host, n_global_segs, seg_offset, full));
    if (world > 1) RET(mm_allreduce_sum_f64_device(c, full, n_global_segs));
    return mm_gate_finalize_device(c, full, n_global_segs, n_blocks, blk_s0_host, blk_s1_host, block_scale, target,
                                   d_out, loudness_gain_host);
}

int mm_finalize(mm_ctx *c, double gain_linear, int use_gain, void *d_out) {
    if (!c || !c->staged) return set_err(c, MM_ERR_STATE, "no staged job");
    return finalize(c, gain_linear, nullptr, use_gain, d_out);
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

// Device-pointer collectives on the context's stream: no host
// staging; the buffers must live on this context's device.  Synchronous on return.
int mm_allreduce_sum_f64_device(mm_ctx *c, double *d_buf, int64_t n) {
    if (!c) return MM_ERR_ARG;
    if (n < 0 || (n > 0 && !d_buf)) return set_err(c, MM_ERR_ARG, "all-reduce: bad buffer");
    if (!c->comm) return set_err(c, MM_ERR_STATE, "communicator not initialised");
    if (n > 0) {
        ncclResult_t r = ncclAllReduce(d_buf, d_buf, (size_t)n, ncclDouble, ncclSum, c->comm, c->stream);
        if (r != ncclSuccess) return set_err(c, MM_ERR_RCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MM_OK;
}

int mm_allgather_f64_device(mm_ctx *c, const double *d_in, double *d_out, int64_t n) {
    if (!c) return MM_ERR_ARG;
    if (n < 0 || (n > 0 && (!d_in || !d_out))) return set_err(c, MM_ERR_ARG, "all-gather: bad buffers");
    if (!c->comm) return set_err(c, MM_ERR_STATE, "communicator not initialised");
    if (n > 0) {
        ncclResult_t r = ncclAllGather(d_in, d_out, (size_t)n, ncclDouble, c->comm, c->stream);
        if (r != ncclSuccess) return set_err(c, MM_ERR_RCCL, "ncclAllGather: %s", ncclGetErrorString(r));
    }
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

// per-stage operators (AME:117-227 one at a time)
#include "ops.hip"
