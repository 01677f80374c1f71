/*
 * mastering.h — C-ABI of the MI355X mastering engine (libmastering_amd.so).
 *
 * Drop-in boundary for the reference's hot path
 *   worker/audio_mastering_engine.py:24  process_audio_from_gcs(gcs_uri, settings)
 * whose per-chunk DSP is AME:48-77 (saturation AME:128, EQ AME:146, width AME:136,
 * int16 quantise AME:123, multiband AME:196) and whose whole-track tail is
 * AME:80-89 (concat, LUFS normalise AME:212, soft limiter AME:224, int16).
 * The Python host (python-audio-mastering_amd/mastering_amd/engine.py) mirrors the
 * reference's `process(...)`/`apply_*` surface and calls these entry points via
 * ctypes.  Plain pointers and sizes only; no torch types.
 *
 * Conventions: every function returns 0 on success and a negative code on error;
 * mm_last_error() then holds a message (per context, NUL terminated).  One context
 * per host thread; a context owns one hipStream_t and its device work buffers.
 * Host-side filter design (EQ/crossover/K-weighting coefficients, compressor
 * max-attenuation tables, state-transition powers, chunk and loudness-block
 * geometry) is done by the caller in f64 with the reference's exact expressions
 * and passed in mm_job, so coefficients are bit-identical to the reference's.
 */
#ifndef MASTERING_AMD_H
#define MASTERING_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MM_OK 0
#define MM_ERR_ARG (-1)
#define MM_ERR_HIP (-2)
#define MM_ERR_RCCL (-3)
#define MM_ERR_STATE (-4)

#define MM_MAX_DIM 8      /* max IIR state dimension per channel (4 biquads) */
#define MM_TILE_POW 8     /* Phi_T^(2^k), k < MM_TILE_POW (tiles per block <= 256) */
#define MM_BLK_POW 65     /* Phi_B^e, e = 0..64 (one look-back window of 64 blocks) */

#define MM_OUT_I16 0 /* interleaved int16 PCM (what AME:89/98 writes)            */
#define MM_OUT_F32 1 /* interleaved f32 = the same PCM / 32768 (decoded form)    */

#define MM_IN_F32 0  /* input: interleaved f32 (decoded PCM16 / 32768)           */
#define MM_IN_I16 1  /* input: interleaved int16 PCM, decoded (x / 32768) on the GPU */

typedef struct mm_ctx mm_ctx;

/* One IIR stage = 1..2 branches of cascaded DF2T biquads fed by the same input.
 * sos[s] = {b0, b1, b2, a1, a2} (a0 == 1), branches laid out branch-major.
 * State-transition matrices of the zero-input recurrence (row-major
 * MM_MAX_DIM x MM_MAX_DIM, only dim x dim used) for the in-kernel tile carry
 * (csrc/lookback.h):
 *   phi_tile_pow[k]  Phi_T^(2^k), Phi_T = A^tile (A: one frame)
 *   phi_blk_pow[e]   Phi_B^e, Phi_B = Phi_T^tpb (tpb = tiles per thread block:
 *                    128 for stereo stages, 256 for mono ones) */
typedef struct mm_iir {
    int32_t nsec;            /* total sections (0 = stage inactive)           */
    int32_t nsec_branch0;    /* sections in branch 0 (rest are branch 1)      */
    int32_t dim;             /* state dim per channel = 2 * nsec              */
    int32_t tpb;             /* tiles per block the block powers were made for */
    int32_t tile;            /* frames per tile the tile powers were made for (the
                                job's tile; K-weighting: a divisor of it, its
                                lanes then run tile/kweight.tile sub-tiles each) */
    int32_t _pad;
    double sos[4][5];
    double phi_tile_pow[MM_TILE_POW][MM_MAX_DIM * MM_MAX_DIM];
    double phi_blk_pow[MM_BLK_POW][MM_MAX_DIM * MM_MAX_DIM];
} mm_iir;

/* Per-band pydub compress_dynamic_range parameters (AME:207-209). */
typedef struct mm_band {
    double thresh_rms;       /* 32768 * 10**(thr/20)                          */
    double attack_frames;    /* attack_ms * (rate/1000.0)                      */
    double release_frames;   /* release_ms * (rate/1000.0)                     */
    int32_t look;            /* int(attack_frames)                             */
    int32_t r0;              /* smallest rms r with M[r] != 0 (32769: none)     */
    const double *lut;       /* host table [32769][4] per integer rms r:
                                {M, M/attack_frames, M/release_frames, 0} with
                                M = (1-1/ratio)*max(20*log(r/thr,10), 0) (0 if r
                                == 0), all in Python float arithmetic          */
    uint64_t lut_key;        /* content key of the M column of lut (nonzero; the
                                context uploads a table only when the key of its
                                cached copy differs).  0: no key, uploaded on
                                every call                                     */
} mm_band;

/* A mastering job for one track (geometry + settings, all host memory). */
typedef struct mm_job {
    int64_t frames_in;       /* decoded input frames N                         */
    int64_t frames_proc;     /* processed frames (pydub 30 s slicing, AME:48-54) */
    int32_t channels;        /* 1 or 2                                         */
    int32_t rate;
    int32_t tile;            /* frames per tile T (divides every full chunk)    */
    int32_t tiles_per_chunk; /* K = chunk_frames / T                            */
    /* settings (AME:58-86) */
    float sat_keep;          /* f32(1 - mix)      (AME:131-134), mix=(s/100)^2 */
    float sat_mix;           /* f32(mix)                                        */
    float sat_drive;         /* f32(1 + 4*mix)                                  */
    int32_t sat_on;          /* saturation != 0                                 */
    double width;            /* AME:60-61                                       */
    int32_t width_on;        /* width != 1.0 and stereo                         */
    int32_t multiband_on;    /* AME:65                                          */
    int32_t lufs_on;         /* settings["lufs"] is not None (AME:84)           */
    int32_t out_kind;        /* MM_OUT_I16 | MM_OUT_F32                         */
    double lufs_target;
    mm_iir eq;               /* AME:154-161, active stages only                */
    mm_iir xover;            /* butter(4) LP250 (branch 0) + HP4000 (branch 1)  */
    mm_iir kweight;          /* pyloudnorm high_shelf then high_pass            */
    mm_band band[3];         /* low / mid / high                                */
    int32_t comp_warmup;     /* super-tiles of speculative warm-up walk before each one */
    int32_t comp_max_iters;  /* cap on fix-up sweeps (exactness check)          */
    int32_t comp_super;      /* frames per super-tile of the envelope solve (rounded to whole tiles) */
    int32_t in_kind;         /* MM_IN_F32 (0) or MM_IN_I16                      */
    /* loudness geometry (pyloudnorm integrated_loudness, block 0.4 s, step 0.1 s) */
    int64_t n_blocks;
    const int64_t *block_lo; /* host [n_blocks] first frame of each block        */
    const int64_t *block_hi; /* host [n_blocks] one-past-last frame (clamped)    */
    int64_t n_segs;          /* distinct boundaries - 1                         */
    const int64_t *seg_bounds; /* host [n_segs+1] sorted distinct block bounds   */
    double block_scale;      /* 1.0 / (0.4 * rate)                              */
    /* apply_saturation (AME:128-134) tabulated on the int16 grid (ABI 4): host
       [65536] f32, entry k + 32768 = the reference's expression evaluated by numpy
       on k / 32768 (AME:121's decoded samples), so the exciter is bit-identical to
       numpy's float32 tanh wherever the input is a decoded int16 (always on the
       reference's path); NULL: the device tanhf (within 2 ulp) everywhere.  Inputs
       off the grid (f32 WAV) always take tanhf. */
    const float *sat_table;
    uint64_t sat_key;        /* content key of sat_table (nonzero; cached per context) */
} mm_job;

typedef struct mm_result {
    double loudness;         /* integrated loudness of the pre-gain mix (LUFS)   */
    double gain_linear;      /* 10 ** ((target - L) / 20), 1.0 if lufs off       */
    int64_t frames_out;      /* == frames_proc                                   */
    int32_t comp_iters;      /* fix-up sweeps the compressor needed              */
    int32_t _pad;
    int64_t comp_active;     /* active (M != 0) frames over the three bands      */
    int64_t comp_walked;     /* frames re-walked by the fix-up sweeps            */
    int64_t comp_jumped;     /* frames the sweeps crossed by exact release jumps */
} mm_result;

/* Geometry of the compressor's envelope solve for a job (mm_solve_geometry: the
   planning arithmetic stage C runs on, computed on the host without a GPU). */
typedef struct mm_solve_geom {
    int32_t tps;             /* tiles per super-tile (a walker's unit)          */
    int32_t tile_rows;       /* M-plane rows per tile: T rounded up to whole walk
                                load blocks (extra rows hold M = 0)            */
    int32_t rows;            /* rows per column: tps * tile_rows + prefetch pad  */
    int32_t walk_block;      /* rows per walk load block (tile_rows is a multiple)  */
    int64_t cols_per_chunk;  /* super-tile columns per chunk (whole blocks of 64) */
    int64_t chunks;
    int64_t chunk_plane_bytes; /* one chunk's part of one band's M plane: walked
                                through 32-bit buffer offsets, < 2^31           */
    int64_t plane_bytes;     /* the three bands' M planes of the whole track     */
    int32_t col_block;       /* columns per comp_rms workgroup / pass-0 wave (64) (ABI 4) */
    int32_t rms_group_tiles; /* tiles per comp_rms workgroup: tps * col_block (ABI 4) */
} mm_solve_geom;

/* ---- context ------------------------------------------------------------ */
int mm_create(int device, mm_ctx **ctx);
int mm_destroy(mm_ctx *ctx);
const char *mm_last_error(mm_ctx *ctx);
int mm_sync(mm_ctx *ctx);
/* ABI version: 2 = mm_band.lut_key and mm_result.comp_jumped (round 3),
   mm_solve_geometry (round 4); 3 = mm_solve_geom.walk_block, the device loudness
   path in composable steps with a world check and the applied gain returned,
   device-pointer collectives (round 5); 4 = mm_job.sat_table / sat_key,
   mm_op_saturation_table, mm_np_sum_f32, mm_check_compressor_math,
   mm_solve_geom.col_block / rms_group_tiles (round 6).  A caller built against an older header must
   refuse a library whose version differs from its own MM_ABI_VERSION. */
#define MM_ABI_VERSION 4
int mm_version(void);
/* The envelope-solve geometry of a job (no context, no GPU).  MM_ERR_ARG if a
   chunk's plane would not fit 32-bit offsets (no track length below 2^31 frames
   at rates up to 192 kHz does) or if comp_super is not 4 tiles (the rms kernel's
   workgroup shape). */
int mm_solve_geometry(const mm_job *job, mm_solve_geom *out);
/* sha256 prefix (16 hex digits) of the sources this library was built from
   (mastering_amd/srcsha.py: the csrc sources and this header) */
const char *mm_source_sha(void);

/* ---- whole chain -------------------------------------------------------- */
/* Host buffers: in = interleaved [frames_in*channels] of job->in_kind (f32 =
 * PCM16/32768, or int16 PCM), out = [frames_proc*channels] of out_kind.
 * Replaces AME:43-98 minus file/GCS IO. */
int mm_master(mm_ctx *ctx, const mm_job *job, const void *in, void *out, mm_result *res);
/* Same, with device-resident input/output (zero-copy; e.g. torch tensors). */
int mm_master_device(mm_ctx *ctx, const mm_job *job, const void *d_in, void *d_out, mm_result *res);

/* A batch of independent tracks (file sharding, BASELINE C3/C5): jobs[i] with
 * device input d_in[i] and output d_out[i]; up to MM_BATCH_STREAMS tracks run at
 * once on streams of their own (child contexts), res[i] (optional) as above. */
#define MM_BATCH_STREAMS 8
int mm_master_batch(mm_ctx *ctx, int n, const mm_job *jobs, const void *const *d_in, void *const *d_out,
                    mm_result *res);

/* ---- WAV files (AME:43 decode, AME:98 export) ------------------------------ */
typedef struct mm_wav_info {
    int64_t frames;          /* whole frames in the data chunk                   */
    int64_t data_offset;     /* byte offset of the samples in the file           */
    int32_t rate;
    int32_t channels;
    int32_t format;          /* 1 = PCM16, 3 = IEEE float32 (EXTENSIBLE resolved) */
    int32_t bits;
} mm_wav_info;
/* Parse a RIFF/WAVE header (PCM16 or float32).  ctx may be NULL (no message). */
int mm_wav_probe(mm_ctx *ctx, const char *path, mm_wav_info *info);
/* Master a WAV file into out_path (PCM16 WAV for MM_OUT_I16, float32 WAV for
 * MM_OUT_F32).  The samples stream from the file through pinned, double-buffered
 * staging into HBM as they are read (PCM16 stays int16 across PCIe and is
 * decoded on the GPU) and the output streams back the same way.  job must be
 * built for the probed frames/rate/channels; its in_kind is ignored (taken from
 * the file). */
int mm_master_wav(mm_ctx *ctx, const mm_job *job, const char *in_path, const char *out_path, mm_result *res);

/* ---- staged entry points (time-sharded multi-GPU, parity probes) -------- */
/* Run AME:48-80 for this job's chunks into the context's int16 mix buffer and
 * the K-weighting per-tile aggregates (state carry-in assumed 0). */
int mm_stage_chunks(mm_ctx *ctx, const mm_job *job, const void *d_in);
/* K-weighting end state of this job's range from a zero start: dim doubles. */
int mm_kweight_range_end(mm_ctx *ctx, double *end_state_host);
/* Per-segment K-weighted energies given a carry-in state (host [dim] or NULL);
 * writes n_segs doubles to host. */
int mm_hop_energies(mm_ctx *ctx, const double *carry_in_host, double *seg_energy_host);
/* Device-resident variant of mm_hop_energies + all-reduce + gating + mm_finalize
 * (VERDICT r03 item 7), in three composable steps (the collective in between may be
 * the library's communicator or torch.distributed over the same device buffer):
 * mm_shard_energies_device zeroes the caller's device vector d_full[n_global_segs]
 * and writes this rank's n_segs energies at seg_offset (synchronous on return);
 * mm_gate_finalize_device gates the whole track on the device (block b: segments
 * [blk_s0[b], blk_s1[b]), energies scaled by block_scale), applies the gain towards
 * `target` LUFS with the limiter, writes this rank's output to d_out and returns
 * {L, applied gain} in loudness_gain[2]. */
int mm_shard_energies_device(mm_ctx *ctx, const double *carry_in_host, int64_t n_global_segs, int64_t seg_offset,
                             double *d_full);
int mm_gate_finalize_device(mm_ctx *ctx, const double *d_full, int64_t n_global_segs, int64_t n_blocks,
                            const int32_t *blk_s0_host, const int32_t *blk_s1_host, double block_scale,
                            double target, void *d_out, double *loudness_gain);
/* All three with the library's communicator between them: `world` is the plan's rank
 * count; world > 1 needs mm_comm_init over exactly `world` ranks on this context
 * (MM_ERR_STATE otherwise: each rank would gate only its own part of the vector). */
int mm_shard_loudness_device(mm_ctx *ctx, const double *carry_in_host, int64_t n_global_segs, int64_t seg_offset,
                             int64_t n_blocks, const int32_t *blk_s0_host, const int32_t *blk_s1_host,
                             double block_scale, double target, int32_t world, void *d_out, double *loudness_gain);
/* Gated loudness from full-track segment energies (host, C restatement of
 * pyloudnorm's gating); returns L via *loudness. */
int mm_gate_loudness(const mm_job *job, const double *seg_energy, double *loudness);
/* numpy's float32 np.sum of x[0..n) (n <= 131072), on the host, through the reduction
 * program the device runs for pyloudnorm's block energies (8192-element buffer
 * chunks, pairwise leaves of <= 128 with eight accumulators): a CPU check that the
 * device sums in numpy's order. */
int mm_np_sum_f32(const float *x, int64_t n, float *out);
/* Verification entry (no reference counterpart): the compressor's device exp10 and
 * exact rms on host arrays of n arguments.  what 0: out[i] = exp10_tab(a[i]) (the
 * gain 10^y of comp_apply, y in [-3, 0]); what 1: out[i] = rms_exact1(a[i], b[i])
 * (comp_rms's audioop.rms: isqrt(floor(S / n)) for integer S = a[i] < 2^53 and
 * n = b[i] >= 1).  Checked by tests/test_compressor_math.py. */
int mm_check_compressor_math(mm_ctx *ctx, int what, const double *a, const double *b, int64_t n, double *out);
/* Apply gain + soft limiter + quantise (AME:84-89) to the staged mix. */
int mm_finalize(mm_ctx *ctx, double gain_linear, int use_gain, void *d_out);
/* Copy the staged pre-gain int16 mix (interleaved) to host (parity probe). */
int mm_read_mix(mm_ctx *ctx, int16_t *host_mix);

/* ---- timing (HIP events on the context stream) -------------------------- */
/* Enable per-kernel event timing; stats are averages over launches. */
int mm_timing(mm_ctx *ctx, int enable);
/* names: '\n'-joined kernel names into buf; ms/launches arrays of cap entries. */
int mm_kernel_stats(mm_ctx *ctx, char *names, int names_cap, double *total_ms, int64_t *launches, int cap);

/* ---- per-stage operators (AME:117-227, one stage at a time) --------------
 * The reference's public DSP helpers as standalone device operators, numpy in /
 * numpy out through host buffers (mastering_amd/ops.py mirrors their Python
 * signatures).  dtype is the sample type of a float input; an f32 input computes
 * in f32 (numpy's dtype rules for the reference's expressions), an f64 one in f64.
 * n counts samples, frames count [frames][channels] rows. */
#define MM_F32 0
#define MM_F64 1
/* audio_segment_to_float_array (AME:117-121): int16 -> f32 / 32768 */
int mm_op_pcm_to_float(mm_ctx *ctx, const int16_t *in, int64_t n, float *out);
/* apply_saturation (AME:128-134); percent != 0 (0 is the identity, no call) */
int mm_op_saturation(mm_ctx *ctx, int dtype, const void *in, int64_t n, double percent, void *out);
/* the same with the int16-grid table of mm_job.sat_table (table: [65536] f32, or
   NULL for the tanhf path): f32 inputs k / 32768 read entry k + 32768, others take
   tanhf; f64 inputs always compute in f64 */
int mm_op_saturation_table(mm_ctx *ctx, int dtype, const void *in, int64_t n, double percent, const float *table,
                           void *out);
/* apply_stereo_width (AME:136-144) on interleaved stereo [frames][2] */
int mm_op_stereo_width(mm_ctx *ctx, int dtype, const void *in, int64_t frames, double width, void *out);
/* float_array_to_audio_segment's samples (AME:123-126): clip, *32768, astype(int16) */
int mm_op_quantize(mm_ctx *ctx, int dtype, const void *in, int64_t n, int16_t *out);
/* soft_limiter (AME:224-227), in place like the reference */
int mm_op_soft_limiter(mm_ctx *ctx, int dtype, void *inout, int64_t n, double threshold);
/* samples * np.float64(gain) -> f64 (AME:222) */
int mm_op_gain(mm_ctx *ctx, int dtype, const void *in, int64_t n, double gain, double *out);
/* scipy.signal.sosfilt of ONE cascade (f->nsec 1..4 sections, all in branch 0,
 * tables for LB tiles/block = 256/channels) over each channel column of
 * [frames][channels], zero initial state; f64 out.  round_f32: every section's
 * output is rounded to f32 (pyloudnorm's lfilter write-backs).  Replaces
 * apply_eq_to_samples / apply_shelf_filter / apply_peak_filter (AME:146-194). */
int mm_op_sosfilt(mm_ctx *ctx, int dtype, const void *in, int64_t frames, int channels, const mm_iir *f,
                  int round_f32, double *out);
/* pyloudnorm Meter(rate).integrated_loudness of samples.mean(axis=1) (AME:213-218).
 * job: channels, frames_proc, kweight (tpb 256), loudness geometry, lufs_target.
 * out[0] = loudness (LUFS), out[1] = 10 ** ((lufs_target - L) / 20). */
int mm_op_loudness(mm_ctx *ctx, const mm_job *job, int dtype, const void *in, double *out);
/* The legacy engine's variants (main.py:94-192, mastering_amd/legacy.py):
 * saturation tanh(x*g)/g with g = 1 + 4*amount/100 (main.py:94-97); limiter
 * |x| > threshold -> tanh(x)*threshold (main.py:189-192); an EQ stage as the
 * parallel mix a*x + c*sosfilt(x) of its butter() filter (main.py:133-154: the
 * a*x product in f32 for f32 samples, numpy's rule), f64 out; and the compressor
 * + overlay on three given int16 band arrays (main.py:156-177, whose mid band is
 * LP4000(HP250(x)) rather than x - lo - hi). */
int mm_op_saturation_legacy(mm_ctx *ctx, int dtype, const void *in, int64_t n, double amount, void *out);
int mm_op_soft_limiter_legacy(mm_ctx *ctx, int dtype, void *inout, int64_t n, double threshold);
int mm_op_sosfilt_mix(mm_ctx *ctx, int dtype, const void *in, int64_t frames, int channels, const mm_iir *f,
                      double a, double c, double *out);
int mm_op_compress_bands(mm_ctx *ctx, const mm_job *job, const int16_t *lo, const int16_t *mid, const int16_t *hi,
                         int16_t *out);
/* apply_multiband_compressor (AME:196-210) on int16 PCM [frames][channels]:
 * job with multiband_on, in_kind MM_IN_I16, EQ/exciter/width/loudness off and one
 * chunk covering the input (tile * tiles_per_chunk >= frames_proc); out has the
 * input's frames (pydub overlay's ms re-slicing is the caller's). */
int mm_op_multiband(mm_ctx *ctx, const mm_job *job, const int16_t *in, int16_t *out);

/* ---- RCCL over xGMI ----------------------------------------------------- */
int mm_comm_unique_id(char id_out[128]);
int mm_comm_init(mm_ctx *ctx, int rank, int nranks, const char id[128]);
int mm_comm_destroy(mm_ctx *ctx);
/* In-place sum all-reduce of n doubles in host memory (staged through HBM). */
int mm_allreduce_sum_f64(mm_ctx *ctx, double *host_buf, int64_t n);
/* All-gather of n doubles per rank: out = [nranks * n]. */
int mm_allgather_f64(mm_ctx *ctx, const double *host_in, double *host_out, int64_t n);
/* The same two collectives on device buffers of this context's device (no host
 * staging; synchronous on return). */
int mm_allreduce_sum_f64_device(mm_ctx *ctx, double *d_buf, int64_t n);
int mm_allgather_f64_device(mm_ctx *ctx, const double *d_in, double *d_out, int64_t n);

#ifdef __cplusplus
}
#endif
#endif
