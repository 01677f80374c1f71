// ops.hip — the reference's per-stage DSP operators (AME:117-227) as standalone
// HIP kernels behind the C-ABI (include/mastering.h, "per-stage operators").
//
// The whole-track chain (mastering.hip) fuses these stages; here each runs on its
// own so that a caller can swap in ONE operator with the reference's signature
// (mastering_amd/ops.py mirrors apply_saturation, apply_eq_to_samples, ...).  The
// numerics follow numpy's dtype rules for the reference's expressions: an f32 input
// computes in f32 with the Python-float constants rounded to f32 (NEP 50 weak
// scalars), an f64 input in f64; scipy's sosfilt/lfilter run in f64.
//
// Included at the end of mastering.hip (one translation unit): the host entry
// points use its context helpers (get_buf, launch, lb_prepare, upload_tables).

namespace mm {

enum PwOp { PW_PCM16, PW_SAT, PW_WIDTH, PW_QUANT, PW_LIMIT, PW_GAIN, PW_MONO, PW_SAT_LEGACY, PW_LIMIT_LEGACY };

struct PwArgs {
    int64_t n;        // elements (frames for WIDTH / MONO)
    const void *in;
    void *out;
    double p0, p1, p2;  // op constants (f64; rounded to f32 inside f32 ops)
    const float *tab;   // PW_SAT on f32: the int16-grid table (mm_op_saturation_table), or null
};

template <typename T>
__device__ __forceinline__ T sat_op(T x, double keep, double mix, double drive, const float *tab) {
    if constexpr (sizeof(T) == 4) {  // f32: (1-mix)*x + mix*tanh(x*(1+4mix)), constants as f32
        float y;
        if (tab && sat_lookup(x, tab, &y)) return y;  // on the int16 grid: numpy's own bits
        const float t = tanhf(__fmul_rn(x, (float)drive));
        return __fadd_rn(__fmul_rn((float)keep, x), __fmul_rn((float)mix, t));
    } else {
        const double t = tanh(__dmul_rn(x, drive));
        return __dadd_rn(__dmul_rn(keep, x), __dmul_rn(mix, t));
    }
}

// soft_limiter (AME:224-227) in the input's dtype; x ** 0.5 is numpy's sqrt fast path
template <typename T>
__device__ __forceinline__ T limit_op(T y, double thr_d) {
    if constexpr (sizeof(T) == 4) {
        const float thr = (float)thr_d;
        const float ay = fabsf(y);
        if (ay > thr) {
            const float d = __fsub_rn(ay, thr);
            const float t = __fdiv_rn(d, 0.02f);
            const float den = sqrt_f32_cr(__fadd_rn(1.0f, __fmul_rn(t, t)));
            const float sg = y > 0 ? 1.0f : (y < 0 ? -1.0f : y);
            y = __fmul_rn(__fadd_rn(thr, __fdiv_rn(d, den)), sg);
        }
        return y;
    } else {
        const double ay = fabs(y);
        if (ay > thr_d) {
            const double d = __dsub_rn(ay, thr_d);
            const double t = __ddiv_rn(d, 0.02);
            const double den = __dsqrt_rn(__dadd_rn(1.0, __dmul_rn(t, t)));
            const double sg = y > 0 ? 1.0 : (y < 0 ? -1.0 : y);
            y = __dmul_rn(__dadd_rn(thr_d, __ddiv_rn(d, den)), sg);
        }
        return y;
    }
}

// one element (or one stereo frame for WIDTH / MONO) per thread, grid-stride
template <int OP, typename T>
__global__ void __launch_bounds__(256) pointwise_kernel(PwArgs a) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        if constexpr (OP == PW_PCM16) {  // audio_segment_to_float_array (AME:117-121)
            const int16_t v = static_cast<const int16_t *>(a.in)[i];
            static_cast<float *>(a.out)[i] = (float)v / 32768.0f;
        } else if constexpr (OP == PW_SAT) {  // apply_saturation (AME:128-134)
            static_cast<T *>(a.out)[i] = sat_op<T>(static_cast<const T *>(a.in)[i], a.p0, a.p1, a.p2, a.tab);
        } else if constexpr (OP == PW_WIDTH) {  // apply_stereo_width (AME:136-144)
            const T *x = static_cast<const T *>(a.in) + 2 * i;
            T *y = static_cast<T *>(a.out) + 2 * i;
            const T l = x[0], r = x[1], w = (T)a.p0;
            T mid, side;
            if constexpr (sizeof(T) == 4) {
                mid = __fdiv_rn(__fadd_rn(l, r), 2.0f);
                side = __fmul_rn(__fdiv_rn(__fsub_rn(l, r), 2.0f), w);
                y[0] = __fadd_rn(mid, side);
                y[1] = __fsub_rn(mid, side);
            } else {
                mid = __ddiv_rn(__dadd_rn(l, r), 2.0);
                side = __dmul_rn(__ddiv_rn(__dsub_rn(l, r), 2.0), w);
                y[0] = __dadd_rn(mid, side);
                y[1] = __dsub_rn(mid, side);
            }
        } else if constexpr (OP == PW_QUANT) {  // float_array_to_audio_segment (AME:123-126)
            static_cast<int16_t *>(a.out)[i] = quantize((double)static_cast<const T *>(a.in)[i]);
        } else if constexpr (OP == PW_LIMIT) {
            static_cast<T *>(a.out)[i] = limit_op<T>(static_cast<const T *>(a.in)[i], a.p0);
        } else if constexpr (OP == PW_GAIN) {  // samples * np.float64 gain -> f64 (AME:222)
            static_cast<double *>(a.out)[i] = __dmul_rn((double)static_cast<const T *>(a.in)[i], a.p0);
        } else if constexpr (OP == PW_SAT_LEGACY) {  // legacy main.py:94-97: tanh(x * g) / g, g = 1 + 4 s / 100
            const T x = static_cast<const T *>(a.in)[i];
            if constexpr (sizeof(T) == 4)
                static_cast<T *>(a.out)[i] = __fdiv_rn(tanhf(__fmul_rn(x, (float)a.p0)), (float)a.p0);
            else
                static_cast<T *>(a.out)[i] = __ddiv_rn(tanh(__dmul_rn(x, a.p0)), a.p0);
        } else if constexpr (OP == PW_LIMIT_LEGACY) {  // legacy main.py:189-192: |x| > thr -> tanh(x) * thr
            T y = static_cast<const T *>(a.in)[i];
            if constexpr (sizeof(T) == 4) {
                if (fabsf(y) > (float)a.p0) y = __fmul_rn(tanhf(y), (float)a.p0);
            } else {
                if (fabs(y) > a.p0) y = __dmul_rn(tanh(y), a.p0);
            }
            static_cast<T *>(a.out)[i] = y;
        } else if constexpr (OP == PW_MONO) {  // samples.mean(axis=1) (AME:215), in T
            const T *x = static_cast<const T *>(a.in) + 2 * i;
            if constexpr (sizeof(T) == 4) static_cast<T *>(a.out)[i] = __fdiv_rn(__fadd_rn(x[0], x[1]), 2.0f);
            else static_cast<T *>(a.out)[i] = __ddiv_rn(__dadd_rn(x[0], x[1]), 2.0);
        }
    }
}

// ---------------------------------------------------------- layout transposes
// natural [N][CH] of T <-> tile-major f64 lines: element (tile g, frame n, channel
// c) at (n*G + g)*CH + c, so a wave's lanes (tile, channel pairs) read 64
// consecutive doubles per step.  A block moves OPS_TILES tiles through LDS so both
// the natural and the tile-major side are coalesced.
constexpr int OPS_TILES = 16;

template <typename T, int CH>
__global__ void __launch_bounds__(256) to_tile_major_kernel(const T *in, double *tm, int64_t N, int64_t G, int Tl) {
    extern __shared__ double tbuf[];  // [OPS_TILES][Tl*CH + 1]
    const int stride = Tl * CH + 1;
    const int64_t g0 = (int64_t)blockIdx.x * OPS_TILES;
    const int64_t f0 = g0 * Tl;
    const int span = OPS_TILES * Tl * CH;
    for (int i = threadIdx.x; i < span; i += blockDim.x) {  // natural side, coalesced
        const int64_t e = f0 * CH + i;
        const int t = i / (Tl * CH), k = i - t * (Tl * CH);
        tbuf[t * stride + k] = e < N * CH ? (double)in[e] : 0.0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < span; i += blockDim.x) {  // tile-major side, coalesced
        const int n = i / (OPS_TILES * CH), r = i - n * (OPS_TILES * CH);
        const int t = r / CH, c = r - t * CH;
        if (g0 + t < G) tm[((int64_t)n * G + g0 + t) * CH + c] = tbuf[t * stride + n * CH + c];
    }
}

template <int CH>
__global__ void __launch_bounds__(256) from_tile_major_kernel(const double *tm, double *out, int64_t N, int64_t G,
                                                              int Tl) {
    extern __shared__ double tbuf[];
    const int stride = Tl * CH + 1;
    const int64_t g0 = (int64_t)blockIdx.x * OPS_TILES;
    const int64_t f0 = g0 * Tl;
    const int span = OPS_TILES * Tl * CH;
    for (int i = threadIdx.x; i < span; i += blockDim.x) {
        const int n = i / (OPS_TILES * CH), r = i - n * (OPS_TILES * CH);
        const int t = r / CH, c = r - t * CH;
        if (g0 + t < G) tbuf[t * stride + n * CH + c] = tm[((int64_t)n * G + g0 + t) * CH + c];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < span; i += blockDim.x) {
        const int64_t e = f0 * CH + i;
        const int t = i / (Tl * CH), k = i - t * (Tl * CH);
        if (e < N * CH) out[e] = tbuf[t * stride + k];
    }
}

// ------------------------------------------------------- generic DF2T cascade
// scipy.signal.sosfilt / lfilter (f64) over each channel line of a tile-major
// array, zero initial state, one launch (lookback.h carry).  R32: the output of
// every section is rounded to f32 before the next one (pyloudnorm writes each
// lfilter pass back into its float32 array, AME:218).
struct IirOpArgs {
    int64_t N, G;
    int T;
    double sos[4][5];
    const double *in;  // tile-major
    double *out;       // tile-major (may alias in: every lane reads its frame before writing it)
    // optional parallel mix of the legacy engine's EQ stages (main.py:133-154):
    // out = a * x + c * filtered, the a * x product in f32 when the samples were f32
    int mix_on, mix_a_f32;
    double mix_a, mix_c;
};

template <int NS, bool R32, bool P2>
__device__ __forceinline__ void iir_op_pass(const IirOpArgs &a, int64_t g, int c, int CH, int len,
                                            double (&z)[NS][2]) {
    const int64_t G = a.G;
    int pn = 0;
    stream<8, 3, double>(
        len, [&](int i) { return a.in[((int64_t)min(i, len - 1) * G + g) * CH + c]; },
        [&](double x) {
            double y = x;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                y = df2t<P2>(y, z[s][0], z[s][1], a.sos[s]);
                if (R32) y = (double)(float)y;
            }
            if (P2) {
                if (a.mix_on) {  // numpy: samples + filtered * c, or samples * a + filtered * c
                    const double ax = a.mix_a == 1.0 ? x
                                      : (a.mix_a_f32 ? (double)__fmul_rn((float)x, (float)a.mix_a) : __dmul_rn(x, a.mix_a));
                    y = __dadd_rn(ax, __dmul_rn(y, a.mix_c));
                }
                a.out[((int64_t)pn * G + g) * CH + c] = y;
            }
            ++pn;
        });
}

template <int NS, int CH, bool R32>
__global__ void __launch_bounds__(LB_THREADS, 2) iir_op_kernel(IirOpArgs a, LbArgs lb) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int TPB = LB_THREADS / CH;
    constexpr int DIM = 2 * NS;
    __shared__ int ticket_slot;
    const int blk = lb_ticket(lb, &ticket_slot);
    const int tid = threadIdx.x;
    const int c = CH == 2 ? (tid & 1) : 0;
    const int t = tid / CH;
    const int64_t g = (int64_t)blk * TPB + t;
    const bool valid = g < a.G;
    const int len = valid ? (int)min((int64_t)a.T, a.N - g * a.T) : 0;
    double zs[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) zs[s][0] = zs[s][1] = 0.0;
    if (valid) iir_op_pass<NS, R32, false>(a, g, c, CH, len, zs);
    double z[DIM], s[DIM], rst[DIM];
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
        z[2 * s_] = zs[s_][0];
        z[2 * s_ + 1] = zs[s_][1];
        rst[2 * s_] = rst[2 * s_ + 1] = 0.0;
    }
    lb_carry<DIM, CH>(lb, blk, t, c, valid, valid && g == 0, rst, z, s, smem);
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
        zs[s_][0] = s[2 * s_];
        zs[s_][1] = s[2 * s_ + 1];
    }
    if (valid) iir_op_pass<NS, R32, true>(a, g, c, CH, len, zs);
}

// Energies of the loudness segments a tile touches (mono tile-major signal; the
// segments are at least one tile long): part[2g], part[2g+1] as kweight_kernel.
__global__ void __launch_bounds__(256) tile_energy_kernel(KwArgs a, const double *tm) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.G) return;
    const int len = (int)min((int64_t)a.T, a.N_proc - g * a.T);
    const int64_t f0 = g * a.T;
    int64_t lo = 0, hi = a.n_segs;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.seg_bounds[mid] <= f0) lo = mid;
        else hi = mid;
    }
    const int64_t seg_end = a.seg_bounds[lo + 1];
    double e0 = 0.0, e1 = 0.0;
    int64_t pf = f0;
    const int64_t G = a.G;
    stream<8, 3, double>(
        len, [&](int i) { return tm[(int64_t)min(i, len - 1) * G + g]; },
        [&](double y) {
            const double e = y * y;
            if (pf < seg_end) e0 += e;
            else e1 += e;
            ++pf;
        });
    a.part[2 * g] = e0;
    a.part[2 * g + 1] = e1;
    a.part_seg[g] = lo;
}

// Three natural int16 band arrays [N][CH] -> the compressor's tile-major band
// planes (int16 pairs, mono R = 0) and per-tile energies E / tail, as the
// crossover kernel leaves them (legacy engine: its bands come from other filters).
template <int CH>
__global__ void __launch_bounds__(256) bands_to_tiles_kernel(const int16_t *lo, const int16_t *mid, const int16_t *hi,
                                                             short2 *plane0, short2 *plane1, short2 *plane2,
                                                             double *tile_e, int64_t N, int64_t G, int Tl,
                                                             int tf0, int tf1, int tf2) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (g >= G) return;
    const int16_t *in = b == 0 ? lo : (b == 1 ? mid : hi);
    short2 *plane = b == 0 ? plane0 : (b == 1 ? plane1 : plane2);
    const int tail_from = b == 0 ? tf0 : (b == 1 ? tf1 : tf2);
    const int len = (int)min((int64_t)Tl, N - g * Tl);
    double E = 0.0, tl = 0.0;
    for (int n = 0; n < len; ++n) {
        const int64_t f = g * Tl + n;
        const int16_t x = in[f * CH];
        const int16_t y = CH == 2 ? in[f * CH + 1] : (int16_t)0;
        plane[(int64_t)n * G + g] = make_short2(x, y);
        const double e = (double)((uint32_t)((int32_t)x * x) + (uint32_t)((int32_t)y * y));
        E += e;
        tl += n >= tail_from ? e : 0.0;
    }
    tile_e[(size_t)(2 * b) * G + g] = E;
    tile_e[(size_t)(2 * b + 1) * G + g] = tl;
}

}  // namespace mm

// ======================================================= host entry points
namespace {

int dtype_size(int dtype) { return dtype == MM_F32 ? 4 : (dtype == MM_F64 ? 8 : 0); }

unsigned pw_blocks(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096)); }

// host in -> device -> kernel -> host out, for the pointwise operators
template <typename Kern>
int run_pointwise(mm_ctx *c, const char *name, Kern k, const void *in, size_t in_bytes, void *out, size_t out_bytes,
                  PwArgs pa) {
    char *din, *dout;
    RET(get_buf(c, "op_in", std::max<size_t>(in_bytes, 1), &din));
    RET(get_buf(c, "op_out", std::max<size_t>(out_bytes, 1), &dout));
    if (in_bytes) HIPCHK(c, hipMemcpyAsync(din, in, in_bytes, hipMemcpyHostToDevice, c->stream));
    pa.in = din;
    pa.out = dout;
    if (pa.n > 0) RET(launch(c, name, k, dim3(pw_blocks(pa.n)), dim3(256), 0, pa));
    if (out_bytes) HIPCHK(c, hipMemcpyAsync(out, dout, out_bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    return MM_OK;
}

#define PW_DISPATCH(OP, dtype, ...)                                                                 \
    ((dtype) == MM_F32 ? run_pointwise(c, #OP, pointwise_kernel<OP, float>, __VA_ARGS__)            \
                       : run_pointwise(c, #OP, pointwise_kernel<OP, double>, __VA_ARGS__))

int check_dtype(mm_ctx *c, int dtype) {
    if (!dtype_size(dtype)) return set_err(c, MM_ERR_ARG, "dtype %d (MM_F32 | MM_F64)", dtype);
    return MM_OK;
}

// natural [N][ch] host samples -> tile-major f64 on the device (tiles of T frames:
// the filter tables' tile, OPS_TILE or the K-weighting sub-tile)
constexpr int OPS_TILE = 125;

int upload_tile_major(mm_ctx *c, int dtype, const void *in, int64_t N, int ch, int64_t G, double **tm, int T) {
    const size_t in_bytes = (size_t)N * ch * dtype_size(dtype);
    char *din;
    RET(get_buf(c, "op_in", std::max<size_t>(in_bytes, 1), &din));
    RET(get_buf(c, "op_tm", (size_t)std::max<int64_t>(G, 1) * T * ch, tm));
    if (in_bytes) HIPCHK(c, hipMemcpyAsync(din, in, in_bytes, hipMemcpyHostToDevice, c->stream));
    const unsigned nb = blocks_for(G, OPS_TILES);
    const size_t lds = ((size_t)OPS_TILES * (T * ch + 1)) * sizeof(double);
    if (dtype == MM_F32) {
        if (ch == 2) return launch(c, "to_tile_major", to_tile_major_kernel<float, 2>, dim3(nb), dim3(256), lds,
                                   (const float *)din, *tm, N, G, T);
        return launch(c, "to_tile_major", to_tile_major_kernel<float, 1>, dim3(nb), dim3(256), lds, (const float *)din,
                      *tm, N, G, T);
    }
    if (ch == 2) return launch(c, "to_tile_major", to_tile_major_kernel<double, 2>, dim3(nb), dim3(256), lds,
                               (const double *)din, *tm, N, G, T);
    return launch(c, "to_tile_major", to_tile_major_kernel<double, 1>, dim3(nb), dim3(256), lds, (const double *)din,
                  *tm, N, G, T);
}

template <int NS, int CH>
int launch_iir_op_ns(mm_ctx *c, bool r32, unsigned nblk, const IirOpArgs &ia, const LbArgs &lb) {
    const size_t lds = lb_lds_bytes<2 * NS, CH>();
    if (r32) return launch(c, "iir_op", iir_op_kernel<NS, CH, true>, dim3(nblk), dim3(LB_THREADS), lds, ia, lb);
    return launch(c, "iir_op", iir_op_kernel<NS, CH, false>, dim3(nblk), dim3(LB_THREADS), lds, ia, lb);
}

template <int CH>
int launch_iir_op(mm_ctx *c, int nsec, bool r32, unsigned nblk, const IirOpArgs &ia, const LbArgs &lb) {
    switch (nsec) {
        case 1: return launch_iir_op_ns<1, CH>(c, r32, nblk, ia, lb);
        case 2: return launch_iir_op_ns<2, CH>(c, r32, nblk, ia, lb);
        case 3: return launch_iir_op_ns<3, CH>(c, r32, nblk, ia, lb);
        default: return launch_iir_op_ns<4, CH>(c, r32, nblk, ia, lb);
    }
}

// cascade f over a tile-major array in place (zero initial state, one line per channel)
int iir_in_place(mm_ctx *c, const mm_iir *f, int64_t N, int ch, int64_t G, double *tm, int round_f32,
                 const double *mix = nullptr, int mix_a_f32 = 0) {
    if (f->nsec < 1 || f->nsec > 4) return set_err(c, MM_ERR_ARG, "nsec %d out of [1, 4]", f->nsec);
    if (f->nsec_branch0 != f->nsec) return set_err(c, MM_ERR_ARG, "the operator filters ONE cascade");
    if (f->tpb != LB_THREADS / ch)
        return set_err(c, MM_ERR_ARG, "tables built for %d tiles/block, need %d", f->tpb, LB_THREADS / ch);
    IirOpArgs ia{};
    ia.N = N;
    ia.G = G;
    ia.T = f->tile;
    for (int s = 0; s < 4; ++s)
        for (int k = 0; k < 5; ++k) ia.sos[s][k] = s < f->nsec ? f->sos[s][k] : 0.0;
    ia.in = tm;
    ia.out = tm;
    if (mix) {
        ia.mix_on = 1;
        ia.mix_a = mix[0];
        ia.mix_c = mix[1];
        ia.mix_a_f32 = mix_a_f32;
    }
    LbArgs lb{};
    RET(upload_tables(c, "op_iir", *f, lb));
    const unsigned nblk = blocks_for(G, LB_THREADS / ch);
    RET(lb_prepare(c, nblk, ch, lb));
    RET(get_buf(c, "op_lb_error", 4, &lb.error));
    HIPCHK(c, hipMemsetAsync(lb.error, 0, 4, c->stream));
    if (ch == 2) RET(launch_iir_op<2>(c, f->nsec, round_f32 != 0, nblk, ia, lb));
    else RET(launch_iir_op<1>(c, f->nsec, round_f32 != 0, nblk, ia, lb));
    unsigned e = 0;
    HIPCHK(c, hipMemcpyAsync(&e, lb.error, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (e) return set_err(c, MM_ERR_STATE, "IIR look-back timed out");
    return MM_OK;
}

}  // namespace

extern "C" {

int mm_op_pcm_to_float(mm_ctx *c, const int16_t *in, int64_t n, float *out) {
    if (!c || (n > 0 && (!in || !out)) || n < 0) return set_err(c, MM_ERR_ARG, "bad arguments");
    HIPCHK(c, hipSetDevice(c->device));
    PwArgs pa{};
    pa.n = n;
    return run_pointwise(c, "op_pcm_to_float", pointwise_kernel<PW_PCM16, float>, in, (size_t)n * 2, out,
                         (size_t)n * 4, pa);
}

int mm_op_saturation_table(mm_ctx *c, int dtype, const void *in, int64_t n, double percent, const float *table,
                           void *out) {
    if (!c || n < 0 || (n > 0 && (!in || !out))) return set_err(c, MM_ERR_ARG, "bad arguments");
    RET(check_dtype(c, dtype));
    HIPCHK(c, hipSetDevice(c->device));
    const double mix = (percent / 100.0) * (percent / 100.0);  // (s/100) ** 2 (Python float)
    PwArgs pa{};
    pa.n = n;
    pa.p0 = 1 - mix;
    pa.p1 = mix;
    pa.p2 = 1 + mix * 4;
    if (table && dtype == MM_F32) {
        float *tab;
        RET(get_buf(c, "op_sat_tab", 65536, &tab));
        HIPCHK(c, hipMemcpyAsync(tab, table, 65536 * sizeof(float), hipMemcpyHostToDevice, c->stream));
        pa.tab = tab;
    }
    const size_t bytes = (size_t)n * dtype_size(dtype);
    return PW_DISPATCH(PW_SAT, dtype, in, bytes, out, bytes, pa);
}

int mm_check_compressor_math(mm_ctx *c, int what, const double *a, const double *b, int64_t n, double *out) {
    if (!c || n < 0 || (what != 0 && what != 1) || (n > 0 && (!a || !out || (what == 1 && !b))))
        return set_err(c, MM_ERR_ARG, "bad arguments");
    if (n == 0) return MM_OK;
    HIPCHK(c, hipSetDevice(c->device));
    double *da, *db, *dout;
    RET(get_buf(c, "cm_a", (size_t)n, &da));
    RET(get_buf(c, "cm_b", (size_t)n, &db));
    RET(get_buf(c, "cm_out", (size_t)n, &dout));
    HIPCHK(c, hipMemcpyAsync(da, a, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
    if (what == 1) HIPCHK(c, hipMemcpyAsync(db, b, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
    RET(launch(c, "comp_math", comp_math_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, what, (const double *)da,
               (const double *)db, n, dout));
    HIPCHK(c, hipMemcpyAsync(out, dout, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MM_OK;
}

int mm_op_saturation(mm_ctx *c, int dtype, const void *in, int64_t n, double percent, void *out) {
    return mm_op_saturation_table(c, dtype, in, n, percent, nullptr, out);
}

int mm_op_stereo_width(mm_ctx *c, int dtype, const void *in, int64_t frames, double width, void *out) {
    if (!c || frames < 0 || (frames > 0 && (!in || !out))) return set_err(c, MM_ERR_ARG, "bad arguments");
    RET(check_dtype(c, dtype));
    HIPCHK(c, hipSetDevice(c->device));
    PwArgs pa{};
    pa.n = frames;
    pa.p0 = width;
    const size_t bytes = (size_t)frames * 2 * dtype_size(dtype);
    return PW_DISPATCH(PW_WIDTH, dtype, in, bytes, out, bytes, pa);
}

int mm_op_quantize(mm_ctx *c, int dtype, const void *in, int64_t n, int16_t *out) {
    if (!c || n < 0 || (n > 0 && (!in || !out))) return set_err(c, MM_ERR_ARG, "bad arguments");
    RET(check_dtype(c, dtype));
    HIPCHK(c, hipSetDevice(c->device));
    PwArgs pa{};
    pa.n = n;
    return PW_DISPATCH(PW_QUANT, dtype, in, (size_t)n * dtype_size(dtype), out, (size_t)n * 2, pa);
}

int mm_op_soft_limiter(mm_ctx *c, int dtype, void *inout, int64_t n, double threshold) {
    if (!c || n < 0 || (n > 0 && !inout)) return set_err(c, MM_ERR_ARG, "bad arguments");
    RET(check_dtype(c, dtype));
    HIPCHK(c, hipSetDevice(c->device));
    PwArgs pa{};
    pa.n = n;
    pa.p0 = threshold;
    const size_t bytes = (size_t)n * dtype_size(dtype);
    return PW_DISPATCH(PW_LIMIT, dtype, inout, bytes, inout, bytes, pa);
}

int mm_op_gain(mm_ctx *c, int dtype, const void *in, int64_t n, double gain, double *out) {
    if (!c || n < 0 || (n > 0 && (!in || !out))) return set_err(c, MM_ERR_ARG, "bad arguments");
    RET(check_dtype(c, dtype));
    HIPCHK(c, hipSetDevice(c->device));
    PwArgs pa{};
    pa.n = n;
    pa.p0 = gain;
    return PW_DISPATCH(PW_GAIN, dtype, in, (size_t)n * dtype_size(dtype), out, (size_t)n * 8, pa);
}

int mm_op_saturation_legacy(mm_ctx *c, int dtype, const void *in, int64_t n, double amount, void *out) {
    if (!c || n < 0 || (n > 0 && (!in || !out))) return set_err(c, MM_ERR_ARG, "bad arguments");
    RET(check_dtype(c, dtype));
    HIPCHK(c, hipSetDevice(c->device));
    PwArgs pa{};
    pa.n = n;
    pa.p0 = 1.0 + (amount / 100.0) * 4.0;  // main.py:95 (Python float)
    const size_t bytes = (size_t)n * dtype_size(dtype);
    return PW_DISPATCH(PW_SAT_LEGACY, dtype, in, bytes, out, bytes, pa);
}

int mm_op_soft_limiter_legacy(mm_ctx *c, int dtype, void *inout, int64_t n, double threshold) {
    if (!c || n < 0 || (n > 0 && !inout)) return set_err(c, MM_ERR_ARG, "bad arguments");
    RET(check_dtype(c, dtype));
    HIPCHK(c, hipSetDevice(c->device));
    PwArgs pa{};
    pa.n = n;
    pa.p0 = threshold;
    const size_t bytes = (size_t)n * dtype_size(dtype);
    return PW_DISPATCH(PW_LIMIT_LEGACY, dtype, inout, bytes, inout, bytes, pa);
}

static int sosfilt_common(mm_ctx *c, int dtype, const void *in, int64_t frames, int channels, const mm_iir *f,
                          int round_f32, const double *mix, double *out) {
    if (!c || !f || frames < 0 || (frames > 0 && (!in || !out))) return set_err(c, MM_ERR_ARG, "bad arguments");
    if (channels != 1 && channels != 2) return set_err(c, MM_ERR_ARG, "channels must be 1 or 2");
    if (frames >= (int64_t)1 << 31) return set_err(c, MM_ERR_ARG, "more than 2^31 frames");
    RET(check_dtype(c, dtype));
    HIPCHK(c, hipSetDevice(c->device));
    if (frames == 0) return MM_OK;
    const int T = f->tile;
    if (T < 1 || T > 512) return set_err(c, MM_ERR_ARG, "filter tables built for %d-frame tiles", T);
    const int64_t G = (frames + T - 1) / T;
    double *tm;
    RET(upload_tile_major(c, dtype, in, frames, channels, G, &tm, T));
    RET(iir_in_place(c, f, frames, channels, G, tm, round_f32, mix, dtype == MM_F32));
    double *dout;
    RET(get_buf(c, "op_out", (size_t)frames * channels, &dout));
    const unsigned nb = blocks_for(G, OPS_TILES);
    const size_t lds = ((size_t)OPS_TILES * (T * channels + 1)) * sizeof(double);
    if (channels == 2)
        RET(launch(c, "from_tile_major", from_tile_major_kernel<2>, dim3(nb), dim3(256), lds, (const double *)tm, dout,
                   frames, G, T));
    else
        RET(launch(c, "from_tile_major", from_tile_major_kernel<1>, dim3(nb), dim3(256), lds, (const double *)tm, dout,
                   frames, G, T));
    HIPCHK(c, hipMemcpyAsync(out, dout, (size_t)frames * channels * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    return MM_OK;
}

int mm_op_sosfilt_mix(mm_ctx *c, int dtype, const void *in, int64_t frames, int channels, const mm_iir *f, double a,
                      double cf, double *out) {
    const double mix[2] = {a, cf};
    return sosfilt_common(c, dtype, in, frames, channels, f, 0, mix, out);
}

// apply_multiband_compressor's compressor + overlay on three given int16 band
// arrays [frames][channels] (the legacy engine's bands, main.py:156-177): the
// chain's stage C on one line (job as for mm_op_multiband; its crossover unused).
int mm_op_compress_bands(mm_ctx *c, const mm_job *j, const int16_t *lo, const int16_t *mid, const int16_t *hi,
                         int16_t *out) {
    if (!c || !j || (j->frames_proc > 0 && (!lo || !mid || !hi || !out))) return set_err(c, MM_ERR_ARG, "bad arguments");
    if (!j->multiband_on || j->eq.nsec || j->sat_on || j->width_on || j->lufs_on)
        return set_err(c, MM_ERR_ARG, "band compressor job: only the multiband stage may be on");
    if (j->frames_in != j->frames_proc || (int64_t)j->tile * j->tiles_per_chunk < j->frames_proc)
        return set_err(c, MM_ERR_ARG, "the operator's chunk must cover the whole input");
    RET(validate(c, j));
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t N = j->frames_proc;
    if (N == 0) return MM_OK;
    const int T = j->tile, ch = j->channels;
    const int64_t G = (N + T - 1) / T;
    const int64_t TG = (int64_t)T * G;
    c->G = G;
    c->job = *j;
    c->staged = false;
    mm_solve_geom sg;
    solve_geometry(j, &sg);  // (checked by stage_compress)
    RET(setup_control(c, blocks_for(G, LB_THREADS / ch), sg.chunks, 3 * sg.chunks * sg.cols_per_chunk * 65 / 64));
    const size_t bytes = (size_t)N * ch * 2;
    char *din;
    RET(get_buf(c, "host_in", 3 * bytes, &din));
    HIPCHK(c, hipMemcpyAsync(din, lo, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(din + bytes, mid, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(din + 2 * bytes, hi, bytes, hipMemcpyHostToDevice, c->stream));
    short2 *bands[3];
    RET(get_buf(c, "band0", TG, &bands[0]));
    RET(get_buf(c, "band1", TG, &bands[1]));
    RET(get_buf(c, "band2", TG, &bands[2]));
    double *tile_e;
    RET(get_buf(c, "comp_tile_e", (size_t)6 * G, &tile_e));
    int tf[3];
    for (int b = 0; b < 3; ++b) {
        const int r = j->band[b].look % T;
        tf[b] = r ? T - r : T;
    }
    const int16_t *p0 = reinterpret_cast<const int16_t *>(din), *p1 = p0 + (size_t)N * ch, *p2 = p1 + (size_t)N * ch;
    if (ch == 2)
        RET(launch(c, "bands_to_tiles", bands_to_tiles_kernel<2>, dim3(blocks_for(G, 256), 3), dim3(256), 0, p0, p1, p2,
                   bands[0], bands[1], bands[2], tile_e, N, G, T, tf[0], tf[1], tf[2]));
    else
        RET(launch(c, "bands_to_tiles", bands_to_tiles_kernel<1>, dim3(blocks_for(G, 256), 3), dim3(256), 0, p0, p1, p2,
                   bands[0], bands[1], bands[2], tile_e, N, G, T, tf[0], tf[1], tf[2]));
    short2 *q2;
    RET(stage_compress(c, j, bands, tile_e, &q2));
    c->mix = q2;
    c->staged = true;
    for (;;) {
        bool converged;
        RET(chain_check(c, &converged));
        if (converged) break;
        RET(comp_sweeps(c, 8));
        RET(comp_back(c));
    }
    return mm_read_mix(c, out);
}

int mm_op_sosfilt(mm_ctx *c, int dtype, const void *in, int64_t frames, int channels, const mm_iir *f,
                  int round_f32, double *out) {
    return sosfilt_common(c, dtype, in, frames, channels, f, round_f32, nullptr, out);
}

// pyloudnorm Meter(rate).integrated_loudness of samples.mean(axis=1) (AME:213-218):
// mono in the input's dtype, K-weighting (f32 write-backs for an f32 input), segment
// energies, gating; out[0] = L, out[1] = 10 ** ((job->lufs_target - L) / 20).
int mm_op_loudness(mm_ctx *c, const mm_job *j, int dtype, const void *in, double *out) {
    if (!c || !j || !out || (j->frames_proc > 0 && !in)) return set_err(c, MM_ERR_ARG, "bad arguments");
    RET(check_dtype(c, dtype));
    const int ch = j->channels;
    const int64_t N = j->frames_proc;
    if (ch != 1 && ch != 2) return set_err(c, MM_ERR_ARG, "channels must be 1 or 2");
    if (N < 1 || N >= (int64_t)1 << 31) return set_err(c, MM_ERR_ARG, "frames %lld out of range", (long long)N);
    if (j->kweight.nsec != 2 || j->kweight.tpb != LB_THREADS) return set_err(c, MM_ERR_ARG, "K-weighting tables");
    if (j->n_segs < 1 || !j->seg_bounds || !j->block_lo || !j->block_hi || j->n_blocks < 1)
        return set_err(c, MM_ERR_ARG, "missing loudness geometry");
    const int T = j->kweight.tile;  // the K-weighting tables' (sub-)tile
    if (T < 1 || T > 512) return set_err(c, MM_ERR_ARG, "K-weighting tables built for %d-frame tiles", T);
    for (int64_t s = 0; s + 1 < j->n_segs; ++s)
        if (std::min<int64_t>(j->seg_bounds[s + 1], N) - j->seg_bounds[s] < T)
            return set_err(c, MM_ERR_ARG, "loudness segment shorter than a tile");
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t G = (N + T - 1) / T;
    const size_t esz = dtype_size(dtype);
    double *tm;
    if (ch == 2) {  // mean(axis=1) on the device, then the mono line
        char *din, *dmono;
        RET(get_buf(c, "op_in", (size_t)N * 2 * esz, &din));
        RET(get_buf(c, "op_mono", (size_t)N * esz, &dmono));
        HIPCHK(c, hipMemcpyAsync(din, in, (size_t)N * 2 * esz, hipMemcpyHostToDevice, c->stream));
        PwArgs pa{};
        pa.n = N;
        pa.in = din;
        pa.out = dmono;
        if (dtype == MM_F32) RET(launch(c, "op_mono", pointwise_kernel<PW_MONO, float>, dim3(pw_blocks(N)), dim3(256), 0, pa));
        else RET(launch(c, "op_mono", pointwise_kernel<PW_MONO, double>, dim3(pw_blocks(N)), dim3(256), 0, pa));
        RET(get_buf(c, "op_tm", (size_t)G * T, &tm));
        const unsigned nb = blocks_for(G, OPS_TILES);
        const size_t lds = ((size_t)OPS_TILES * (T + 1)) * sizeof(double);
        if (dtype == MM_F32)
            RET(launch(c, "to_tile_major", to_tile_major_kernel<float, 1>, dim3(nb), dim3(256), lds,
                       (const float *)dmono, tm, N, G, T));
        else
            RET(launch(c, "to_tile_major", to_tile_major_kernel<double, 1>, dim3(nb), dim3(256), lds,
                       (const double *)dmono, tm, N, G, T));
    } else {
        RET(upload_tile_major(c, dtype, in, N, 1, G, &tm, T));
    }
    RET(iir_in_place(c, &j->kweight, N, 1, G, tm, dtype == MM_F32));
    // segment energies -> gating on the device (gate.hip)
    double *part, *seg, *gout;
    int64_t *part_seg;
    RET(get_buf(c, "op_part", (size_t)G * 2, &part));
    RET(get_buf(c, "op_part_seg", (size_t)G, &part_seg));
    RET(get_buf(c, "op_seg", (size_t)j->n_segs, &seg));
    RET(get_buf(c, "op_gate", 2, &gout));
    mm_job saved = c->job;  // upload_geometry reads the context's job
    c->job = *j;
    const int rc = upload_geometry(c);
    c->job = saved;
    RET(rc);
    KwArgs ka{};
    ka.N_proc = N;
    ka.G = G;
    ka.T = T;
    ka.Gt = G;
    ka.sub = 1;
    ka.ch = 1;
    ka.n_segs = j->n_segs;
    ka.seg_bounds = c->seg_bounds_dev;
    ka.part = part;
    ka.part_seg = part_seg;
    RET(launch(c, "op_tile_energy", tile_energy_kernel, dim3(blocks_for(G, 256)), dim3(256), 0, ka, (const double *)tm));
    RET(launch(c, "op_seg_reduce", seg_reduce_kernel, dim3(blocks_for(j->n_segs, 4)), dim3(256), 0, ka, seg));
    GateArgs ga{};
    ga.n_blocks = j->n_blocks;
    ga.blk_s0 = c->blk_s0;
    ga.blk_s1 = c->blk_s1;
    ga.seg = seg;
    ga.scale = j->block_scale;
    ga.target = j->lufs_target;
    ga.out = gout;
    RET(gate_launch(c, ga, 1));
    HIPCHK(c, hipMemcpyAsync(out, gout, 2 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    return MM_OK;
}

// apply_multiband_compressor (AME:196-210) on int16 PCM [frames][channels]: the
// chain's crossover + compressor + overlay stages on ONE line (the job's chunk
// covers the whole input; its EQ, exciter, width and loudness must be off).  The
// output has the input's frame count (pydub overlay's ms re-slicing is applied by
// the caller, mastering_amd/ops.py).
int mm_op_multiband(mm_ctx *c, const mm_job *j, const int16_t *in, int16_t *out) {
    if (!c || !j || (j->frames_proc > 0 && (!in || !out))) return set_err(c, MM_ERR_ARG, "bad arguments");
    if (!j->multiband_on || j->eq.nsec || j->sat_on || j->width_on || j->lufs_on || j->in_kind != MM_IN_I16)
        return set_err(c, MM_ERR_ARG, "multiband operator job: only the multiband stage may be on (int16 input)");
    if (j->frames_in != j->frames_proc) return set_err(c, MM_ERR_ARG, "frames_in != frames_proc");
    if ((int64_t)j->tile * j->tiles_per_chunk < j->frames_proc)
        return set_err(c, MM_ERR_ARG, "the operator's chunk must cover the whole input");
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t N = j->frames_proc;
    if (N == 0) return MM_OK;
    const size_t bytes = (size_t)N * j->channels * 2;
    char *din;
    RET(get_buf(c, "host_in", bytes, &din));
    HIPCHK(c, hipMemcpyAsync(din, in, bytes, hipMemcpyHostToDevice, c->stream));
    RET(stage_chunks(c, j, din));
    return mm_read_mix(c, out);
}

}  // extern "C"
