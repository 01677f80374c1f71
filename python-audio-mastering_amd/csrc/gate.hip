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
    double *zl;             // scratch [2 n_blocks]: z_j, then l_j (gate_blocks_kernel)
};

constexpr int GATE_THREADS = 1024;

// z_j and l_j of every block, one thread per block (the segment sum in segment
// order, as the host restatement): the gate itself then streams them coalesced.
// (Round 5 computed them inside the one-workgroup gate, a dependent chain of
// segment loads per block and thread: 220 us for a 2-hour track, 13 us for C2.)
constexpr int GATE_BLK_THREADS = 256;
__global__ void __launch_bounds__(GATE_BLK_THREADS) gate_blocks_kernel(GateArgs a) {
    const int64_t j = (int64_t)blockIdx.x * GATE_BLK_THREADS + threadIdx.x;
    if (j >= a.n_blocks) return;
    const int32_t s0 = a.blk_s0[j], s1 = a.blk_s1[j];
    double acc = 0.0;
    for (int32_t s = s0; s < s1; ++s) acc += a.seg[s];
    const double z = a.scale * acc;
    a.zl[j] = z;
    a.zl[a.n_blocks + j] = -0.691 + 10.0 * log10(z);
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

// One workgroup per track over its blocks' (z, l) from gate_blocks_kernel: thread t
// sums blocks t, t + 1024, ... in order, then the fixed-order reduction.
__global__ void __launch_bounds__(GATE_THREADS) gate_kernel(GateArgs a) {
    __shared__ double rs[GATE_THREADS / 64];
    __shared__ long long rc[GATE_THREADS / 64];
    const int t = threadIdx.x;
    const int64_t j0 = a.trk_blk ? a.trk_blk[blockIdx.x] : 0;
    const int64_t j1 = a.trk_blk ? a.trk_blk[blockIdx.x + 1] : a.n_blocks;
    double *out = a.out + 2 * blockIdx.x;
    const double *zv = a.zl, *lv = a.zl + a.n_blocks;
    double sum = 0.0;
    long long cnt = 0;
#pragma unroll 8
    for (int64_t j = j0 + t; j < j1; j += GATE_THREADS) {
        const double z = zv[j], l = lv[j];
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
#pragma unroll 8
    for (int64_t j = j0 + t; j < j1; j += GATE_THREADS) {
        const double z = zv[j], l = lv[j];
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
