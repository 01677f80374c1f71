// gate.hip — pyloudnorm's gated integrated loudness and the normalisation gain,
// on the device, so the chain runs without a host round trip (AME:212-222).
//
// pyloudnorm 0.1.1 Meter.integrated_loudness (mono, channel gain 1):
//   z_j   = (1/(0.4 rate)) * sum of K-weighted y^2 over block j (0.4 s, 0.1 s hop)
//   l_j   = -0.691 + 10 log10(z_j)
//   abs   : J_a = { j : l_j >= -70 }
//   rel   : Gamma_r = -0.691 + 10 log10(mean_{J_a} z) - 10
//   final : J_g = { j : l_j > Gamma_r and l_j > -70 },  L = -0.691 + 10 log10(mean_{J_g} z)
//           (nan_to_num: an empty J_g gives z = 0 -> L = -inf)
// AME:219-222: gain = 10 ** ((target - L) / 20).
// Block energies are sums of the 0.1 s segment energies kweight_kernel produced;
// the per-block sum runs in segment order like the host restatement
// (mm_gate_loudness); the reductions over blocks are tree-ordered (the result
// differs from a sequential sum in the last bits only).
#include "common.h"

namespace mm {

struct GateArgs {
    int64_t n_blocks;
    const int32_t *blk_s0;  // first segment of block j
    const int32_t *blk_s1;  // one past its last segment
    const double *seg;      // segment energies
    double scale;           // 1 / (0.4 rate)
    double target;          // LUFS target
    double *out;            // [0] = L, [1] = gain
    const int64_t *trk_blk; // fused batch: block b gates track b's blocks [trk_blk[b], trk_blk[b+1])
                            // into out[2b], out[2b+1]; null: one track, blocks [0, n_blocks)
};

constexpr int GATE_THREADS = 1024;

__device__ __forceinline__ double gate_block_z(const GateArgs &a, int64_t j) {
    double acc = 0.0;
    for (int s = a.blk_s0[j]; s < a.blk_s1[j]; ++s) acc += a.seg[s];
    return a.scale * acc;
}

// sum and count over the block, result broadcast to every thread: a fixed-order
// butterfly within each wave, then the waves' partials in order (deterministic)
__device__ __forceinline__ void gate_reduce(double &sum, long long &cnt, double *rs, long long *rc) {
    const int t = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o);
        cnt += __shfl_xor(cnt, o);
    }
    if ((t & 63) == 0) {
        rs[t >> 6] = sum;
        rc[t >> 6] = cnt;
    }
    __syncthreads();
    sum = 0.0;
    cnt = 0;
#pragma unroll
    for (int w = 0; w < GATE_THREADS / 64; ++w) {
        sum += rs[w];
        cnt += rc[w];
    }
    __syncthreads();
}

constexpr int GATE_CACHE = 4;  // block energies a thread keeps between the two gates

__global__ void __launch_bounds__(GATE_THREADS) gate_kernel(GateArgs a) {
    __shared__ double rs[GATE_THREADS / 64];
    __shared__ long long rc[GATE_THREADS / 64];
    const int t = threadIdx.x;
    const int64_t j0 = a.trk_blk ? a.trk_blk[blockIdx.x] : 0;
    const int64_t j1 = a.trk_blk ? a.trk_blk[blockIdx.x + 1] : a.n_blocks;
    double *out = a.out + 2 * blockIdx.x;
    double zc[GATE_CACHE], lc[GATE_CACHE];  // the thread's first blocks (a 5-min track: 3 each)
    double sum = 0.0;
    long long cnt = 0;
    // the cached blocks first, their segment loads issued together (one latency
    // instead of a dependent chain per block: the kernel is a single workgroup)
    int32_t b0[GATE_CACHE], b1[GATE_CACHE];
#pragma unroll
    for (int k = 0; k < GATE_CACHE; ++k) {
        const int64_t j = j0 + t + (int64_t)k * GATE_THREADS;
        b0[k] = j < j1 ? a.blk_s0[j] : 0;
        b1[k] = j < j1 ? a.blk_s1[j] : 0;
    }
    // (a 0.4 s block spans 4 segments of 0.1 s, 5 at a ragged end: the first four
    // loads of every block are issued without a wait)
    double sv[GATE_CACHE][4];
#pragma unroll
    for (int k = 0; k < GATE_CACHE; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) sv[k][u] = b0[k] + u < b1[k] ? a.seg[b0[k] + u] : 0.0;
#pragma unroll
    for (int k = 0; k < GATE_CACHE; ++k) {
        double acc = 0.0;  // segment order, as gate_block_z
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (b0[k] + u < b1[k]) acc += sv[k][u];
        for (int s_ = b0[k] + 4; s_ < b1[k]; ++s_) acc += a.seg[s_];
        zc[k] = a.scale * acc;
    }
#pragma unroll
    for (int k = 0; k < GATE_CACHE; ++k) {
        const int64_t j = j0 + t + (int64_t)k * GATE_THREADS;
        lc[k] = -0.691 + 10.0 * log10(zc[k]);
        if (j < j1 && lc[k] >= -70.0) {
            sum += zc[k];
            ++cnt;
        }
    }
    int i = GATE_CACHE;
    for (int64_t j = j0 + t + (int64_t)GATE_CACHE * GATE_THREADS; j < j1; j += GATE_THREADS, ++i) {
        const double z = gate_block_z(a, j);
        const double l = -0.691 + 10.0 * log10(z);
        if (l >= -70.0) {
            sum += z;
            ++cnt;
        }
    }
    gate_reduce(sum, cnt, rs, rc);
    const double mean_abs = cnt ? sum / (double)cnt : __longlong_as_double(0x7ff8000000000000LL);
    const double gamma_r = -0.691 + 10.0 * log10(mean_abs) - 10.0;
    sum = 0.0;
    cnt = 0;
    i = 0;
    for (int64_t j = j0 + t; j < j1; j += GATE_THREADS, ++i) {
        double z, l;
        if (i < GATE_CACHE) {
            z = zc[i];
            l = lc[i];
        } else {
            z = gate_block_z(a, j);
            l = -0.691 + 10.0 * log10(z);
        }
        if (l > gamma_r && l > -70.0) {
            sum += z;
            ++cnt;
        }
    }
    gate_reduce(sum, cnt, rs, rc);
    if (t == 0) {
        const double zavg = cnt ? sum / (double)cnt : 0.0;
        const double L = -0.691 + 10.0 * log10(zavg);
        out[0] = L;
        out[1] = pow(10.0, (a.target - L) / 20.0);
    }
}

}  // namespace mm
