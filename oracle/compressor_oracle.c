/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle for the multiband compressor band loop.
 * Nothing in the product path (python-audio-mastering_amd/) may link or call this.
 *
 * Restates pydub 0.25.1 `effects.compress_dynamic_range` (third-party, not vendored
 * in /root/reference; called at worker/audio_mastering_engine.py:207-209) together
 * with the CPython 3.10 `audioop.rms` / `audioop.mul` semantics it relies on.
 * Parity at this boundary is "unpinned" by the reference's own tests (it has none);
 * the restatement is cross-checked against stdlib audioop in tests/test_oracle.py
 * and against the pure-Python pydub-structured loop in tests/golden/make_golden.py.
 *
 * Semantics (per frame i of a band segment with `frames` frames, `ch` channels):
 *   window      = frames [max(0, i-look), i)            (get_sample_slice, excl. i)
 *   rms         = (unsigned)sqrt(sum_sq / nsamples)      (audioop.rms, 0 if empty)
 *   dbo         = rms==0 ? 0 : max(20*log(rms/thr)/log(10), 0)   (ratio_to_db)
 *   M           = (1 - 1/ratio) * dbo
 *   if rms > thr && att <= M:  att = min(att + M/attack_frames, M)
 *   else:                       att = max(att - M/release_frames, 0)
 *   if att != 0: sample = floor(clamp(sample * 10**(-att/20)))      (audioop.mul)
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* Python float ops are IEEE double with no contraction; keep it that way. */
#pragma STDC FP_CONTRACT OFF

static double py_ratio_to_db(double ratio) {
    volatile double l10 = log(10.0);
    return 20.0 * (log(ratio) / l10);
}

static int16_t audioop_mul_sample(int16_t x, double factor) {
    double val = (double)x * factor;
    if (val > 32767.0) val = 32767.0;
    else if (val < -32768.0 + 1.0) val = -32768.0;
    return (int16_t)(int)floor(val);
}

/*
 * in/out: interleaved int16 [frames * ch]. `out` may alias `in` only if the
 * caller does not need `in` afterwards (the window reads the ORIGINAL samples,
 * so we never alias internally). Optional att_trace (frames doubles) receives
 * the attenuation after the update of each frame.
 */
int oracle_compress_band(const int16_t *in, int16_t *out, int64_t frames, int ch,
                         double threshold_db, double ratio, double attack_ms,
                         double release_ms, double rate, double *att_trace) {
    const double max_amp = 32768.0; /* pydub max_possible_amplitude for width 2 */
    const double thresh_rms = max_amp * pow(10.0, threshold_db / 20.0);
    const double attack_frames = attack_ms * (rate / 1000.0);
    const double release_frames = release_ms * (rate / 1000.0);
    const int64_t look = (int64_t)attack_frames;
    double att = 0.0;
    /* running exact sum of squares over the window (int64 is exact here) */
    int64_t sum = 0;
    for (int64_t i = 0; i < frames; ++i) {
        /* window [lo, i) */
        int64_t lo = i - look;
        if (lo < 0) lo = 0;
        if (i > 0) {
            const int16_t *f = in + (i - 1) * ch;
            for (int c = 0; c < ch; ++c) sum += (int64_t)f[c] * f[c];
        }
        if (i - look - 1 >= 0) {
            const int16_t *f = in + (i - look - 1) * ch;
            for (int c = 0; c < ch; ++c) sum -= (int64_t)f[c] * f[c];
        }
        int64_t nsamp = (i - lo) * ch;
        unsigned int rms = 0;
        if (nsamp > 0) rms = (unsigned int)sqrt((double)sum / (double)nsamp);
        double dbo;
        if (rms == 0) {
            dbo = 0.0;
        } else {
            double db = py_ratio_to_db((double)rms / thresh_rms);
            dbo = db > 0.0 ? db : (db == 0.0 ? db : 0.0);
        }
        double max_att = (1.0 - (1.0 / ratio)) * dbo;
        double inc = max_att / attack_frames;
        double dec = max_att / release_frames;
        if ((double)rms > thresh_rms && att <= max_att) {
            att = att + inc;
            if (max_att < att) att = max_att;
        } else {
            att = att - dec;
            if (0.0 > att) att = 0.0;
        }
        if (att_trace) att_trace[i] = att;
        const int16_t *src = in + i * ch;
        int16_t *dst = out + i * ch;
        if (att != 0.0) {
            double g = pow(10.0, (-att) / 20.0);
            for (int c = 0; c < ch; ++c) dst[c] = audioop_mul_sample(src[c], g);
        } else {
            for (int c = 0; c < ch; ++c) dst[c] = src[c];
        }
    }
    return 0;
}

/* Only the attenuation trajectory (used by the coalescence study and tests). */
int oracle_compress_trace(const int16_t *in, int64_t frames, int ch,
                          double threshold_db, double ratio, double attack_ms,
                          double release_ms, double rate, double att0,
                          int64_t start, int64_t stop, double *att_trace) {
    const double max_amp = 32768.0;
    const double thresh_rms = max_amp * pow(10.0, threshold_db / 20.0);
    const double attack_frames = attack_ms * (rate / 1000.0);
    const double release_frames = release_ms * (rate / 1000.0);
    const int64_t look = (int64_t)attack_frames;
    double att = att0;
    for (int64_t i = start; i < stop && i < frames; ++i) {
        int64_t lo = i - look;
        if (lo < 0) lo = 0;
        int64_t sum = 0;
        for (int64_t j = lo; j < i; ++j)
            for (int c = 0; c < ch; ++c) sum += (int64_t)in[j * ch + c] * in[j * ch + c];
        int64_t nsamp = (i - lo) * ch;
        unsigned int rms = 0;
        if (nsamp > 0) rms = (unsigned int)sqrt((double)sum / (double)nsamp);
        double dbo = 0.0;
        if (rms != 0) {
            double db = py_ratio_to_db((double)rms / thresh_rms);
            dbo = db > 0.0 ? db : (db == 0.0 ? db : 0.0);
        }
        double max_att = (1.0 - (1.0 / ratio)) * dbo;
        if ((double)rms > thresh_rms && att <= max_att) {
            att = att + max_att / attack_frames;
            if (max_att < att) att = max_att;
        } else {
            att = att - max_att / release_frames;
            if (0.0 > att) att = 0.0;
        }
        att_trace[i - start] = att;
    }
    return 0;
}
