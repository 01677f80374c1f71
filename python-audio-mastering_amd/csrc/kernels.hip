// kernels.hip — pointwise / integer kernels of the chain (gfx950): pydub's
// int16 arithmetic helpers used by the compressor, and the final stage
// (gain + soft limiter + int16/f32 output).  The recurrences live in iir.hip
// (EQ, crossover, K-weighting) and compressor.hip (envelope).
#include "common.h"

namespace mm {

// audioop.mul of one int16 sample (pydub compressor output, AME:207-209).
__device__ __forceinline__ int16_t audioop_mul(int16_t x, double g) {
    // audioop's "v > 32767 -> 32767; v < -32767 -> -32768; floor(v)" equals
    // floor(v) clamped to [-32768, 32767] (v in (-32768, -32767) floors to
    // -32768 too); min/max instead of branches
    // (clamping the floored integer: the bounds are integers, so clamp(floor(v)) ==
    // floor(clamp(v)); |x g| <= 32768 here, inside v_cvt_i32_f64's range)
    const int32_t i = (int32_t)floor((double)x * g);
    return (int16_t)min(max(i, -32768), 32767);
}

__device__ __forceinline__ int16_t sat16(int32_t v) {
    return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
}

// ------------------------------------------------ stage E: gain + limiter
// AME:84-89: y = int16/32768 (f32); with a loudness target the gain is an
// np.float64 so y*gain, the soft limiter and the clip run in f64; without
// one they run in f32.  Output natural interleaved layout.  A block handles
// FIN_TILES tiles: the tile-major mix is read coalesced into LDS, then written
// out frame-major coalesced.  16 tiles per block (round 5: 0.045 -> 0.040 ms on
// C2 against 32; 64 took 0.072).
#ifndef MM_FIN_TILES
#define MM_FIN_TILES 16
#endif
constexpr int FIN_TILES = MM_FIN_TILES;

__device__ __forceinline__ double limiter64(double y) {
    double ay = fabs(y);
    if (ay > 0.98) {
        double d = ay - 0.98;
        double t = d / 0.02;
        double den = sqrt(1.0 + t * t);
        double v = 0.98 + d / den;
        double sg = y > 0 ? 1.0 : (y < 0 ? -1.0 : y);
        y = v * sg;
    }
    return y;
}

__device__ __forceinline__ float limiter32(float y) {
    float ay = fabsf(y);
    if (ay > 0.98f) {
        float d = __fsub_rn(ay, 0.98f);
        float t = __fdiv_rn(d, 0.02f);
        float den = sqrt_f32_cr(__fadd_rn(1.0f, __fmul_rn(t, t)));
        float v = __fadd_rn(0.98f, __fdiv_rn(d, den));
        float sg = y > 0 ? 1.0f : (y < 0 ? -1.0f : y);
        y = __fmul_rn(v, sg);
    }
    return y;
}

template <int CH>
__global__ void __launch_bounds__(256) finalize_kernel(FinArgs a) {
    extern __shared__ short2 lds[];  // [FIN_TILES][T+1]
    const int T = a.T;
    const int stride = T + 1;
    const int64_t g0 = (int64_t)blockIdx.x * FIN_TILES;
    const int ntile = (int)min((int64_t)FIN_TILES, a.G - g0);
    if (a.ctl) {  // chain tail: this block's slice of the control block past the readback area
        const int64_t words = (a.ctl_bytes - a.rb_area) / 4, per = (words + gridDim.x - 1) / gridDim.x;
        unsigned *z = reinterpret_cast<unsigned *>(a.ctl + a.rb_area);
        const int64_t end = min(words, (int64_t)(blockIdx.x + 1) * per);
        for (int64_t i = (int64_t)blockIdx.x * per + threadIdx.x; i < end; i += blockDim.x) z[i] = 0u;
    }
    for (int i = threadIdx.x; i < T * FIN_TILES; i += blockDim.x) {
        const int n = i / FIN_TILES, t = i % FIN_TILES;
        if (t < ntile) lds[t * stride + n] = a.mix[(int64_t)n * a.Gs + a.g_off + g0 + t];
    }
    __syncthreads();
    const int64_t f_base = g0 * T;
    const int nf = (int)min((int64_t)ntile * T, a.N_proc - f_base);
    const double gain = a.gain_dev ? *a.gain_dev : a.gain;
    // frame i of the block = (tile t, offset n); t, n advance incrementally
    // (no division per frame: the stride 256 is below T * FIN_TILES)
    int t = (int)((unsigned)threadIdx.x / (unsigned)T), n = (int)threadIdx.x - t * T;
    const int dt = 256 / T, dn = 256 - dt * T;
    for (int i = threadIdx.x; i < nf; i += 256) {
        const short2 q = lds[t * stride + n];
        const int16_t qq[2] = {q.x, q.y};
        int16_t o[2];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const float y = (float)qq[c] / 32768.0f;
            o[c] = a.use_gain ? quantize(limiter64((double)y * gain)) : quantize((double)limiter32(y));
        }
        const int64_t f = f_base + i;
        if (a.out_kind == 0) {
            int16_t *out = reinterpret_cast<int16_t *>(a.out);
            if (CH == 2) *reinterpret_cast<short2 *>(out + 2 * f) = make_short2(o[0], o[1]);
            else out[f] = o[0];
        } else {
            float *out = reinterpret_cast<float *>(a.out);
            if (CH == 2) *reinterpret_cast<float2 *>(out + 2 * f) = make_float2(o[0] * (1.0f / 32768.0f), o[1] * (1.0f / 32768.0f));
            else out[f] = o[0] * (1.0f / 32768.0f);
        }
        t += dt;
        n += dn;
        if (n >= T) {
            n -= T;
            ++t;
        }
    }
    if (a.ctl) {  // chain tail: the last block out hands the readback area to the host
        // No fences: the words copied were written by earlier launches (visible at the
        // launch boundary), and the other blocks' only reads of the area (the gain)
        // completed before their stores above, which precede their count.  (A
        // device-scope fence per block writes back L2 on this part: finalize 0.165
        // against 0.040 ms.)  The area zeroed last includes the done counters.
        __shared__ int last;
        __syncthreads();  // (every read of the device gain in this block is done)
        if (threadIdx.x == 0) {
            const unsigned k = blockIdx.x % FIN_DONE_LINES, lines = min(gridDim.x, (unsigned)FIN_DONE_LINES);
            const unsigned need = (gridDim.x - k + FIN_DONE_LINES - 1) / FIN_DONE_LINES;  // blocks on counter k
            last = atomicAdd(a.done + 32 * k, 1u) == need - 1 &&
                   atomicAdd(a.done + 32 * FIN_DONE_LINES, 1u) == lines - 1;
        }
        __syncthreads();
        if (last) {
            const unsigned *src = reinterpret_cast<const unsigned *>(a.ctl);
            unsigned *dst = reinterpret_cast<unsigned *>(a.rb_host);
            for (int i = threadIdx.x; i < a.rb_bytes / 4; i += blockDim.x) dst[i] = src[i];
            __syncthreads();
            unsigned *z = reinterpret_cast<unsigned *>(a.ctl);
            for (int64_t i = threadIdx.x; i < a.rb_area / 4; i += blockDim.x) z[i] = 0u;
        }
    }
}

// copy the tile-major mix to natural interleaved int16 (parity probe)
__global__ void mix_to_natural_kernel(const short2 *mix, int16_t *out, int64_t G, int T, int64_t N, int ch) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= N) return;
    int64_t g = f / T, n = f - g * T;
    short2 q = mix[n * G + g];
    if (ch == 2) {
        out[2 * f] = q.x;
        out[2 * f + 1] = q.y;
    } else {
        out[f] = q.x;
    }
}

}  // namespace mm
