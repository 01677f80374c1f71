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
// Block energies z_j: exactly pyloudnorm's (kw_blocks_kernel, numpy's float32
// reduction order) on the single-track and fused-batch chains; sums of 0.1 s
// segment energies (f64) on the time-sharded and per-stage paths (gate_blocks).
// The reductions over blocks are tree-ordered (the result differs from numpy's
// pairwise mean in the last bits only: ~1e-16 of the gain).
#include <type_traits>

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

// ---- exact block energies (pyloudnorm's z_j bit for bit) ----------------------
// pyloudnorm computes z_j = (1/(0.4 rate)) * np.sum(np.square(x[lo:hi])) with x the
// float32 K-weighted line: the squares are f32, np.sum is numpy's float32 add.reduce
// and the product with the Python float is f32 (NEP 50).  numpy reduces a contiguous
// array in buffer chunks of 8192 elements, res = 0 then res += pairwise(chunk), where
// pairwise(m) is: m < 8 a sequential sum; m <= 128 eight interleaved accumulators
// r[j] over elements j, j+8, ... combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then
// the m % 8 tail in order; else pairwise(n2) + pairwise(m - n2), n2 = m/2 - (m/2)%8.
// The host turns that recursion into a program per distinct block length
// (mastering.hip pw_build, checked against np.sum on the CPU through mm_np_sum_f32):
//   ints [0..4]  nleaves, nnodes, nlevels, nchunks, root value (-1: empty sum)
//   then chunk_leaf[nchunks + 1], leaf_off[nleaves], leaf_len[nleaves],
//   node_a[nnodes], node_b[nnodes], level_node[nlevels + 1]
// values 0..nleaves-1 are the leaves, nleaves + k node k = val[a] + val[b]; nodes are
// sorted by height so each level only reads earlier ones.
struct KbArgs {
    const float *sq;          // f32 squares of the K-weighted line, tile g at g * TP (kweight_kernel<true>)
    int T, TP;                // frames per tile, padded tile stride (a multiple of 4)
    int64_t n_blocks;
    const int64_t *blk_lo;    // first frame of each block
    const int32_t *blk_n;     // its length
    const int32_t *blk_prog;  // its program (int offset into prog)
    const int32_t *prog;
    float scale;              // f32(1 / (0.4 rate))
    double *zl;               // [2 n_blocks]: z_j, then l_j (read by gate_kernel)
    int stage_floats, nvals, pints;  // dynamic LDS layout (kb_lds_bytes: nvals = both value buffers), pints % 4 == 0
};
constexpr int KB_CHUNK = 8192;   // numpy's reduction buffer (elements)
constexpr int KB_VMAX = 1536;    // leaves + nodes of one block (76 800 frames at 192 kHz: 1199)
constexpr int KB_PMAX = 2560;    // ints of one program (192 kHz: 2430); programs start 16-byte aligned
constexpr int KB_THREADS = 256;
constexpr int KB_LD = 9;         // 16-byte loads per thread per chunk: padded tile quads of the tiles a
                                 // chunk spans, (8191 / T + 2) * ceil(T / 4) <= 2304 (host-checked)

// Dynamic LDS of kw_blocks_kernel: the staged chunk (frame order), the leaf/node
// values (two buffers), the program.
// chunk index -> LDS word: 8 words of padding per 128 frames (a wave's 16 leaves
// start 128 frames apart: with the padding their 8-word groups fill 64 banks twice)
__host__ __device__ constexpr int kb_pad(int i) { return i + ((i >> 7) << 3); }
__host__ __device__ constexpr int kb_lds_bytes(int stage_floats, int nvals, int pints) {
    return stage_floats * 4 + ((nvals + 3) / 4 * 4) * 4 + pints * 4;
}

// Persistent workgroups: workgroup w of XCD x (x = w % 8) takes the blocks
// x per + w/8, + grid/8, ... of its XCD's contiguous range (neighbouring blocks'
// windows overlap 3/4: the re-reads hit that XCD's L2).  The blocks' chunks
// (8192 frames, numpy's buffers) form one stream over all the workgroup's blocks
// with KB_RING chunks' 16-byte loads in flight (a ring of register buffers).  Per
// chunk the tiles' padded runs are copied to LDS as they lie in memory (a plain
// 16-byte copy); eight lanes per leaf run numpy's eight accumulators, walking the
// frames' word addresses; per block the
// program's levels combine the leaves in numpy's order.  A block's program (one
// per block length) stays in LDS while the next block has the same.
#ifndef MM_KB_RING
#define MM_KB_RING 1
#endif
constexpr int KB_RING = MM_KB_RING;  // chunks in flight per workgroup (1-3)
__global__ void __launch_bounds__(KB_THREADS) kw_blocks_kernel(KbArgs a) {
    extern __shared__ __attribute__((aligned(16))) float kb_smem[];
    __shared__ int kb_prog_cur;
    const int tid = threadIdx.x;
    float *el = kb_smem;
    float *val = kb_smem + a.stage_floats;
    int32_t *P = reinterpret_cast<int32_t *>(val + (a.nvals + 3) / 4 * 4);
    const int64_t nbk = a.n_blocks;
    const int64_t per = (nbk + 7) / 8;
    const int xcd = (int)(blockIdx.x % 8), nslot = (int)(gridDim.x / 8);
    const int64_t jb = xcd * per + blockIdx.x / 8, je = min((int64_t)(xcd + 1) * per, nbk);
    if (jb >= je) return;  // (workgroup-uniform)
    const int T = a.T, TP = a.TP, Q4 = a.TP / 4;  // frames per tile, padded tile stride, its 16-byte quads
    const float4 *sq4 = reinterpret_cast<const float4 *>(a.sq);
    float4 *el4 = reinterpret_cast<float4 *>(el);
    if (tid == 0) kb_prog_cur = -1;
    float4 buf[KB_RING][KB_LD];
    int g_nld[KB_RING], g_fb[KB_RING];  // per buffer: quads loaded; the chunk's first frame's row in its tile
    // the stream's next chunk: (block lj, chunk lc)
    int64_t lj = jb;
    int lc = 0;
    int64_t lF0 = a.blk_lo[lj];
    int ln = a.blk_n[lj];
    while (ln <= 0 && lj < je) {
        lj += nslot;
        if (lj < je) lF0 = a.blk_lo[lj], ln = a.blk_n[lj];
    }
    // the chunk's padded tile runs [tA, tB] land in LDS as they lie in memory: quad
    // L of the run is LDS quad L (a plain 16-byte copy); frame u of the run (u = row
    // + T * tile) is LDS word (u / T) TP + u % T
    auto issue = [&](auto B) __attribute__((always_inline)) {  // the stream's next chunk into buffer B
        constexpr int b = decltype(B)::value;
        if (lj >= je) return;
        const int m = min(KB_CHUNK, ln - lc * KB_CHUNK);
        const int64_t F0 = lF0 + (int64_t)lc * KB_CHUNK;
        const int64_t tA = F0 / T;
        const int nld = (int)((F0 + m - 1) / T - tA + 1) * Q4;
        g_nld[b] = nld;
        g_fb[b] = (int)(F0 - tA * T);
        const float4 *base = sq4 + tA * Q4;
#pragma unroll
        for (int r = 0; r < KB_LD; ++r) buf[b][r] = base[min(tid + r * KB_THREADS, nld - 1)];
        if (++lc * KB_CHUNK >= ln) {  // advance (blocks without frames have no chunks)
            lc = 0;
            for (lj += nslot; lj < je; lj += nslot) {
                lF0 = a.blk_lo[lj];
                ln = a.blk_n[lj];
                if (ln > 0) break;
            }
        }
    };
    auto copy = [&](auto B) __attribute__((always_inline)) {  // buffer B -> LDS
        constexpr int b = decltype(B)::value;
#pragma unroll
        for (int r = 0; r < KB_LD; ++r) {
            const float4 v = buf[b][r];
            float *d = el + 4 * min(tid + r * KB_THREADS, g_nld[b] - 1);
            if (tid + r * KB_THREADS < g_nld[b]) d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
        }
    };
    issue(std::integral_constant<int, 0>{});
    if constexpr (KB_RING > 1) issue(std::integral_constant<int, 1 % KB_RING>{});
    if constexpr (KB_RING > 2) issue(std::integral_constant<int, 2 % KB_RING>{});
    int ring = 0;  // the buffer holding the next chunk to sum
    int vb = 0;    // val double buffer: the levels of block j read val[vb] while block j+1 fills the other
    for (int64_t j = jb; j < je; j += nslot, vb ^= 1) {
        const int pj = a.blk_prog[j];
        __syncthreads();  // (everyone is done with P, el and this val buffer's previous block)
        if (pj != kb_prog_cur) {  // a new program into LDS (the device buffer is padded by pints ints)
            const int4 *src = reinterpret_cast<const int4 *>(a.prog + pj);
            int4 *dst = reinterpret_cast<int4 *>(P);
            for (int i = tid; i < a.pints / 4; i += KB_THREADS) dst[i] = src[i];
            __syncthreads();
            if (tid == 0) kb_prog_cur = pj;
        }
        const int nl = P[0], nn = P[1], nlev = P[2], nch = P[3], root = P[4];
        const int32_t *chunk_leaf = P + 5, *loff = chunk_leaf + nch + 1, *llen = loff + nl, *na = llen + nl,
                      *nb = na + nn, *lvl = nb + nn;
        float *V = val + vb * ((a.nvals + 1) / 2);  // (nvals counts both buffers)
        for (int c = 0; c < nch; ++c) {
            const int l0 = chunk_leaf[c], l1 = chunk_leaf[c + 1];
            int fb;
#ifndef MM_KB_NOCOPY  // (ablation builds: timing only)
            if (KB_RING == 1 || ring == 0) copy(std::integral_constant<int, 0>{}), fb = g_fb[0];
            else if (KB_RING == 2 || ring == 1) copy(std::integral_constant<int, 1 % KB_RING>{}), fb = g_fb[1 % KB_RING];
            else copy(std::integral_constant<int, 2 % KB_RING>{}), fb = g_fb[2 % KB_RING];
#else
            fb = g_fb[0];
#endif
            __syncthreads();
            if (KB_RING == 1 || ring == 0) issue(std::integral_constant<int, 0>{});
            else if (KB_RING == 2 || ring == 1) issue(std::integral_constant<int, 1 % KB_RING>{});
            else issue(std::integral_constant<int, 2 % KB_RING>{});
            ring = ring == KB_RING - 1 ? 0 : ring + 1;
            // chunk frame i -> LDS word
            auto word = [&](int i) __attribute__((always_inline)) {
                const int u = i + fb, t = u / T;
                return t * TP + (u - t * T);
            };
            const int q = tid & 7;  // accumulator q of the leaf (eight lanes per leaf)
#ifdef MM_KB_NOLEAF  // (ablation builds: timing only)
            if (l1 < 0)
#endif
            for (int li = l0 + (tid >> 3); li < l1; li += KB_THREADS / 8) {
                const int off = loff[li] - c * KB_CHUNK, len = llen[li];
                float res;
                if (len < 8) {  // (a chunk shorter than 8: numpy's sequential sum)
                    res = el[word(off)];
                    for (int i = 1; i < len; ++i) res = __fadd_rn(res, el[word(off + i)]);
                } else {
                    // this lane's frames off + q + 8g: word addresses advance by 8, and by
                    // the tile padding TP - T when they cross into the next tile
                    const int u0 = off + q + fb, t0 = u0 / T;
                    int row = u0 - t0 * T, w = t0 * TP + row;
                    auto next = [&]() __attribute__((always_inline)) {
                        row += 8;
                        w += 8;
                        if (row >= T) {
                            row -= T;
                            w += TP - T;
                        }
                    };
                    float r;
                    const int full = len - (len & 7);
                    if (full == 128) {  // the common leaf: every read issued at once
                        int ad[16];
#pragma unroll
                        for (int g = 0; g < 16; ++g) {
                            ad[g] = w;
                            next();
                        }
                        float v[16];
#pragma unroll
                        for (int g = 0; g < 16; ++g) v[g] = el[ad[g]];
                        r = v[0];
#pragma unroll
                        for (int g = 1; g < 16; ++g) r = __fadd_rn(r, v[g]);
                    } else {
                        r = el[w];
                        for (int i = 8; i < full; i += 8) {
                            next();
                            r = __fadd_rn(r, el[w]);
                        }
                    }
                    // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)): f32 addition commutes, so every
                    // lane of the eight ends with the same bits
                    r = __fadd_rn(r, __shfl_xor(r, 1));
                    r = __fadd_rn(r, __shfl_xor(r, 2));
                    res = __fadd_rn(r, __shfl_xor(r, 4));
                    for (int i = full; i < len; ++i) res = __fadd_rn(res, el[word(off + i)]);
                }
                if (q == 0) V[li] = res;
            }
            __syncthreads();  // (the next chunk overwrites el; the levels read V)
        }
#ifndef MM_KB_NOLEVEL  // (ablation builds: timing only)
        for (int L = 0; L < nlev; ++L) {
            for (int k = lvl[L] + tid; k < lvl[L + 1]; k += KB_THREADS) V[nl + k] = __fadd_rn(V[na[k]], V[nb[k]]);
            __syncthreads();
        }
#endif
        if (tid == 0) {
            const float sm = root < 0 ? 0.0f : V[root];
            const double z = (double)__fmul_rn(a.scale, sm);
            a.zl[j] = z;
            a.zl[nbk + j] = -0.691 + 10.0 * log10(z);
        }
    }
}

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
