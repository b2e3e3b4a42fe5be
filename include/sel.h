/*
 * sel.h — C ABI of libsel.so, the MI355X (gfx950) kernels behind the
 * denoise-training hot path of s194584/dl-speech-enhancement.
 *
 * Conventions (all entry points):
 *   - every pointer is caller-owned DEVICE memory, contiguous, fp32 unless the
 *     name says otherwise; the library never allocates device memory — scratch
 *     comes in through (ws, ws_bytes) sized by the matching *_workspace() call;
 *   - work is only enqueued on `stream` (no host sync); functions are stateless
 *     and reentrant after sel_init();
 *   - return 0 on success or a negative SEL_ERR_* code; sel_last_error() gives
 *     a thread-local message.  Nothing throws across the ABI.
 *
 * The reference has no native API (it is pure PyTorch); each entry point names
 * the reference function it replaces (file:line under the reference root).
 */
#ifndef SEL_H_
#define SEL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* sel_stream_t; /* == hipStream_t */

enum {
  SEL_OK = 0,
  SEL_ERR_ARG = -1,         /* bad shape / size / pointer */
  SEL_ERR_HIP = -2,         /* HIP runtime error */
  SEL_ERR_UNSUPPORTED = -3, /* legal for the reference but not implemented */
  SEL_ERR_WORKSPACE = -4,   /* workspace too small */
  SEL_ERR_STATE = -5        /* sel_init() not called / failed */
};

enum { SEL_LOG_E = 0, SEL_LOG_2 = 1, SEL_LOG_10 = 2 };

/* ---- library ---------------------------------------------------------- */
int sel_init(void);                 /* uploads FFT twiddle tables; idempotent */
const char* sel_last_error(void);   /* thread-local, never NULL */
int sel_version(void);

/* ---- STFT magnitude: losses/stft_loss.py:19-35 (stft) ------------------
 * x (B,T) -> mag (B, F, K), F = 1 + T/hop, K = n_fft/2 + 1.
 * torch.stft semantics: center=True, reflect pad n_fft/2, periodic window of
 * win_length zero-padded centred to n_fft, onesided, unnormalised;
 * mag = sqrt(max(re^2 + im^2, pow_floor)).  n_fft in {256..4096}, power of 2. */
int sel_stft_mag_fwd(const float* x, int64_t B, int64_t T, int n_fft, int hop,
                     int win_length, const float* window, float pow_floor,
                     float* mag, sel_stream_t stream);
/* grad: g_x (B,T) from g_mag (B,F,K).  Overwrites g_x. */
size_t sel_stft_bwd_workspace(int64_t B, int64_t T, int n_fft, int hop, int win_length);
int sel_stft_mag_bwd(const float* x, int64_t B, int64_t T, int n_fft, int hop,
                     int win_length, const float* window, float pow_floor,
                     const float* g_mag, float* g_x, void* ws, size_t ws_bytes,
                     sel_stream_t stream);

/* ---- SC + log-magnitude reductions on magnitudes -----------------------
 * losses/stft_loss.py:45-56 (SpectralConvergenceLoss), :66-77 (LogSTFTMagnitudeLoss).
 * sums (3 doubles, device) = { sum (y-x)^2, sum y^2, sum |ln y - ln x| } over n. */
size_t sel_mag_pair_workspace(int64_t n);
int sel_mag_pair_sums(const float* x_mag, const float* y_mag, int64_t n,
                      double* sums, void* ws, size_t ws_bytes, sel_stream_t stream);
/* coef (device, 4 floats) = {a, b, c, d}:
 *   g_x = a*(x - y) + b*sign(ln x - ln y)/x
 *   g_y = c*(y - x) + d*y + b*sign(ln y - ln x)/y      (g_y may be NULL)  */
int sel_mag_pair_bwd(const float* x_mag, const float* y_mag, int64_t n, const float* coef,
                     float* g_x, float* g_y, sel_stream_t stream);

/* ---- fused STFT loss for one resolution: losses/stft_loss.py:100-117 ---
 * Computes both STFTs per frame in LDS, never writes magnitudes.
 * sums (3 doubles) as sel_mag_pair_sums.  bwd: coef (device, 2 floats) = {a, b},
 * g_x = dL/dx through g_xmag = a*(xm - ym) + b*sign(ln xm - ln ym)/xm. */
size_t sel_stft_loss_workspace(int64_t B, int64_t T, int n_fft, int hop, int win_length);
int sel_stft_loss_fwd(const float* x, const float* y, int64_t B, int64_t T, int n_fft,
                      int hop, int win_length, const float* window, double* sums,
                      void* ws, size_t ws_bytes, sel_stream_t stream);
int sel_stft_loss_bwd(const float* x, const float* y, int64_t B, int64_t T, int n_fft,
                      int hop, int win_length, const float* window, const float* coef,
                      float* g_x, void* ws, size_t ws_bytes, sel_stream_t stream);
/* Finishing arithmetic on device (no host sync): from sums -> out2 = {sc, mag}
 * and, for the backward, coef = {a, b, c, d} (see sel_mag_pair_bwd) given the
 * upstream grads *g_sc, *g_mag (device scalars; NULL = zero). */
int sel_stft_loss_finish(const double* sums, int64_t n, float* out2, sel_stream_t stream);
int sel_stft_loss_coef(const double* sums, int64_t n, const float* g_sc, const float* g_mag,
                       float* coef, sel_stream_t stream);

/* ---- log-mel: losses/mel_loss.py:74-94 (MelSpectrogram.forward) -------
 * x (B,T) -> out (B, n_mels, F).  melmat (K, n_mels) is the module buffer;
 * krange (n_mels int2) = nonzero bin range [lo,hi) of each filter, mrange (K int2)
 * = filters touching each bin, both derived from melmat by the host. */
int sel_logmel_fwd(const float* x, int64_t B, int64_t T, int n_fft, int hop,
                   int win_length, const float* window, const float* melmat,
                   const int32_t* krange, int n_mels, float eps, int log_kind,
                   float* out, sel_stream_t stream);
/* L1 between two (n) tensors: losses/mel_loss.py:153 F.l1_loss -> out (1 float, mean). */
size_t sel_l1_workspace(int64_t n);
int sel_l1_mean(const float* a, const float* b, int64_t n, float* out, void* ws,
                size_t ws_bytes, sel_stream_t stream);
/* backward of  g * mean|logmel(x) - ref|  w.r.t. x, or of sum(logmel(x)*g_out) when
 * ref == NULL (then `g_out` (B,M,F) is the upstream gradient, g_scale unused).
 * With ref != NULL: g_out is logmel(x) from the forward and the upstream of each
 * element is (*g_scale) * g_mul * sign(g_out - ref)  (g_mul = 1/N for a mean).
 * Overwrites g_x. */
size_t sel_logmel_bwd_workspace(int64_t B, int64_t T, int n_fft, int hop, int win_length);
int sel_logmel_bwd(const float* x, int64_t B, int64_t T, int n_fft, int hop,
                   int win_length, const float* window, const float* melmat,
                   const int32_t* krange, const int32_t* mrange, int n_mels, float eps, int log_kind,
                   const float* g_out, const float* ref, const float* g_scale, float g_mul,
                   float* g_x, void* ws, size_t ws_bytes, sel_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SEL_H_ */
