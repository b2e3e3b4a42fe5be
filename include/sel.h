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
/* tuning knobs for A/B runs inside one process (keys 0..127; key 0: conv fwd
 * kernel variant, 0 = built-in heuristic); returns the previous value, -1 for a
 * key out of range (the call then changes nothing). */
int sel_tune(int key, int value);
/* current value of a tuning knob, read-only (-1 for a key out of range). */
int sel_tune_get(int key);
/* diagnostics: out[2i], out[2i+1] = raw_buffer_load_b64 of x at byte offset 4i
 * (i < n-1) through the STFT kernels' buffer resource (spectral.hip fetch_frame);
 * mode 0: elements taken as scalars, mode 1: __builtin_bit_cast of the vector
 * elements (miscompiled by ROCm 7.2 clang: element 0 twice) */
int sel_probe_buffer_b64(const float* x, int n, int mode, float* out, sel_stream_t stream);
/* measurement: copy n16 16-byte elements (float4) src -> dst with `blocks`
 * workgroups striding over the buffer (the HBM copy-rate denominator of the
 * STFT roofline in bench.py) */
int sel_probe_copy_f4(const void* src, void* dst, int64_t n16, int blocks, sel_stream_t stream);

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
 * upstream grads *g_sc, *g_mag (device scalars; NULL = zero).  n = the
 * element count of the log-magnitude mean, or 0: read it from sums[3] (a
 * 4-element sums array whose count was all-reduced on device by a
 * data-parallel caller). */
int sel_stft_loss_finish(const double* sums, int64_t n, float* out2, sel_stream_t stream);
int sel_stft_loss_coef(const double* sums, int64_t n, const float* g_sc, const float* g_mag,
                       float* coef, sel_stream_t stream);

/* ---- log-mel: losses/mel_loss.py:74-94 (MelSpectrogram.forward) -------
 * x (B,T) -> out (B, n_mels, F).  melmat (K, n_mels) is the module buffer;
 * krange (n_mels int2) = nonzero bin range [lo,hi) of each filter, mrange (K int2)
 * = filters touching each bin, both derived from melmat by the host.
 * 0 < n_mels <= n_fft/2 + 12 (SEL_ERR_UNSUPPORTED otherwise, as the backward). */
int sel_logmel_fwd(const float* x, int64_t B, int64_t T, int n_fft, int hop,
                   int win_length, const float* window, const float* melmat,
                   const int32_t* krange, int n_mels, float eps, int log_kind,
                   float* out, sel_stream_t stream);
/* ---- power-mel: mel_spectrogram.py:38-44 (torchaudio MelSpectrogram(48000), eval Mel-L1) --
 * x (B,T) -> out (B, n_mels, F), F = 1 + T/hop: |STFT|^power (center/reflect, periodic
 * window of win_length centred in n_fft, onesided) @ fb (K, n_mels), K = n_fft/2 + 1.
 * n_fft even, n_fft/2 <= 512 with prime factors in {2,3,5} (n_fft 400 -> 200 = 4*2*5*5).
 * krange as for sel_logmel_fwd.  Forward only (an eval metric). */
int sel_power_mel_fwd(const float* x, int64_t B, int64_t T, int n_fft, int hop, int win_length,
                      const float* window, const float* fb, const int32_t* krange, int n_mels, float power,
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
/* Fused log-mel L1 (mel_loss.py:151-154): *loss = mean |logmel(x) - logmel(y)|
 * over (B, n_mels, F), and, when g_x != NULL, g_x = d loss / d x for a unit
 * upstream (the backward scales it by the upstream gradient): one launch per
 * resolution computes y's and x's log-mels per frame position and x's adjoint
 * (k_mel_l1), then the overlap-add.  mrange / krange as for sel_logmel_bwd.
 * 0 < n_mels <= n_fft/2 + 12.  ws >= sel_mel_l1_workspace(...). */
size_t sel_mel_l1_workspace(int64_t B, int64_t T, int n_fft, int hop, int win_length);
int sel_mel_l1_fwd_grad(const float* x, const float* y, int64_t B, int64_t T, int n_fft, int hop,
                        int win_length, const float* window, const float* melmat, const int32_t* krange,
                        const int32_t* mrange, int n_mels, float eps, int log_kind, float* loss, float* g_x,
                        void* ws, size_t ws_bytes, sel_stream_t stream);
size_t sel_logmel_bwd_workspace(int64_t B, int64_t T, int n_fft, int hop, int win_length);
int sel_logmel_bwd(const float* x, int64_t B, int64_t T, int n_fft, int hop,
                   int win_length, const float* window, const float* melmat,
                   const int32_t* krange, const int32_t* mrange, int n_mels, float eps, int log_kind,
                   const float* g_out, const float* ref, const float* g_scale, float g_mul,
                   float* g_x, void* ws, size_t ws_bytes, sel_stream_t stream);

/* ---- AudioDec conv stack: layers/conv_layer.py, residual_unit.py -------
 * Every conv of the generator is lowered to ONE primitive over channels-last
 * activations (rows = B*T flat, row pitch = channels):
 *   out[m, n] = epi( sum_{k<K} sum_{c<C} Wp[n][k][c] * act(in[row(m,k), c]) )
 *   row(m,k) = b*T + t + k*dil - pad  (t = m % T, b = m / T); rows outside the
 *   sample read 0 (SEL_PAD_ZERO) or clamp to the sample (SEL_PAD_REPLICATE);
 *   act = ELU (alpha 1) when in_elu, else identity;
 *   epi(v) = (v + bias[n % bias_period]) * (aux ? ELU'(aux[m,n]) : 1) + (res ? res[m,n] : 0).
 * Strided convs (encoder down-sampling, conv_layer.py:109-150 with stride s) run
 * as a 3-tap conv on the phase-expanded input (B, T/s, s*Cin); transposed convs
 * (conv_layer.py:153-191) as a 2-tap replicate-padded conv producing
 * (B, T, s*Cout) = (B, T*s, Cout).  Weights are repacked on device each step
 * (sel_pack_weight) and weight gradients unpacked (sel_unpack_wgrad). */
enum { SEL_F32 = 0, SEL_BF16 = 1 };
enum { SEL_PAD_ZERO = 0, SEL_PAD_REPLICATE = 1 };
enum {
  SEL_PACK_FWD = 0,          /* Conv1d W[Cout][Cin][K]          -> Wp[Cout][K][Cin] */
  SEL_PACK_FWD_STRIDED = 1,  /* Conv1d W[Cout][Cin][2s], stride s -> Wp[Cout][3][s*Cin] */
  SEL_PACK_CONVT = 2         /* ConvTranspose1d W[Cin][Cout][2s]  -> Wp[s*Cout][2][Cin] */
};

typedef struct sel_conv_desc {
  int64_t rows;       /* B*T */
  int32_t T;          /* rows per sample */
  int32_t C, N;       /* in / out channels */
  int32_t K, dil, pad;
  int32_t pad_mode;   /* SEL_PAD_* */
  int32_t in_elu;
  int32_t bias_period;/* 0: no bias */
} sel_conv_desc;

/* which kernel instance a bf16 launch uses (for profiling tags); has_epilogue:
 * the launch passes aux and/or res (the thin kernel's epilogue-prefetch variant):
 * ((BM*1000 + BN)*10 + WAVES_M)*10 + KMAX for the tiled kernel,
 * 900000000 + K for the warp-specialised kernel,
 * 1000000000 + E*500000000 + ((R/32*1000 + C)*1000 + N)*10 + K for the
 * weight-stationary thin kernel (E = epilogue-prefetch instance),
 * or -1 for the generic kernel */
int sel_conv_fwd_kernel_id(const sel_conv_desc* d, int in_dtype, int out_dtype, int has_epilogue);
int sel_conv_fwd(const sel_conv_desc* d, int in_dtype, int out_dtype, const void* in,
                 const void* wpack, const float* bias, const void* aux, const void* res,
                 void* out, sel_stream_t stream);
/* Fused residual unit forward (replaces the two sel_conv_fwd calls of
 * models/autoencoder/modules/residual_unit.py:43-46, conv_layer.py:19-23 + :139-142):
 * h = conv1(ELU(x)) [saved for the backward] and out = x + conv1x1(ELU(h)), bf16,
 * C = N in {32, 64} -- or 128 where conv1 alone runs on the (16, 128)
 * k_conv_wss tile (T = 2000-like sequences, >= 65536 rows; sel_tune key 69 = 1
 * turns that off) -- K = 7, causal zero pad; d1 describes conv1 (in_elu = 1).
 * Returns SEL_ERR_UNSUPPORTED for any other shape. */
int sel_resunit_fwd(const sel_conv_desc* d1, int dtype, const void* x, const void* w1pack, const float* b1,
                    const void* w2pack, const float* b2, void* h, void* out, sel_stream_t stream);
/* Fused residual-unit backward at 32 channels (replaces the two adjoint
 * primitive calls of residual_unit.py:43-46's backward): gh = (W2^T g) * ELU'(h),
 * gx = conv1^T(gh) * ELU'(x) + g; d1 is conv1's forward descriptor, wd1/wd2 the
 * dgrad-packed weights (sel_pack_dgrad); gh may be NULL. */
int sel_resunit_bwd(const sel_conv_desc* d1, int dtype, const void* g, const void* h, const void* x,
                    const void* wd1pack, const void* wd2pack, void* gh, void* gx, sel_stream_t stream);
/* The same backward WITH both weight gradients of the unit, in one launch (the
 * residual units whose weights train; 32 channels): gx as sel_resunit_bwd, and
 * per-block fp32 partials of conv1 (part1: nsplit x 32*7*32 packed [N][K][C],
 * then nsplit x 32 bias column sums of gh) and of the 1x1 (part2: nsplit x
 * 32*32, then nsplit x 32 of g).  nsplit = sel_resunit_wgrad_splits(d1, dtype)
 * (a negative code for an unsupported shape); reduce the partials with
 * sel_wgrad_finish_many (kind SEL_PACK_FWD, k 7 and 1). */
int sel_resunit_wgrad_splits(const sel_conv_desc* d1, int dtype);
int sel_resunit_bwd_wgrad(const sel_conv_desc* d1, int dtype, const void* g, const void* h, const void* x,
                          const void* wd1pack, const void* wd2pack, void* gx, float* part1, float* part2,
                          int nsplit, sel_stream_t stream);
/* weight/bias gradient of the same primitive: gwpack[N][K][C] (fp32) and, when
 * gbias != NULL, gbias[bias_period] = sum over rows and phases of gout. */
size_t sel_conv_wgrad_workspace(const sel_conv_desc* d);
int sel_conv_wgrad(const sel_conv_desc* d, int dtype, const void* gout, const void* in,
                   float* gwpack, float* gbias, void* ws, size_t ws_bytes, sel_stream_t stream);
/* sel_conv_wgrad with the weight gradient written straight into the torch layout
 * of the layer's fp32 weight (kind/cout/cin/k/stride as in sel_pack_weight): the
 * unpack is fused into the final reduction pass. */
int sel_conv_wgrad_unpacked(const sel_conv_desc* d, int dtype, const void* gout, const void* in, int kind,
                            int cout, int cin, int k, int stride, float* gw, float* gbias, void* ws,
                            size_t ws_bytes, sel_stream_t stream);
/* Deferred weight gradients (one reduction launch for many layers):
 * sel_conv_wgrad_partials runs only the split-row partial kernel of
 * sel_conv_wgrad into ws (same plan, same partials) and returns the split count
 * in *nsplit; sel_wgrad_finish_many then reduces up to any number of such
 * workspaces in one launch per 24 jobs, with the arithmetic of the per-layer
 * reduction passes (same bits), unpacking into the torch layout (kind >= 0) or
 * writing the packed form (kind < 0).  `jobs` is a HOST array. */
typedef struct sel_wgrad_job {
  const float* part;  /* the workspace of sel_conv_wgrad_partials */
  float* gw;          /* weight gradient (torch layout when kind >= 0) */
  float* gb;          /* bias gradient (bias_period entries) or NULL */
  int64_t nw;         /* N * K * C (packed weight elements) */
  int32_t nsplit, N, bias_period, kind, cout, cin, k, stride;
} sel_wgrad_job;
int sel_conv_wgrad_partials(const sel_conv_desc* d, int dtype, const void* gout, const void* in, int want_bias,
                            void* ws, size_t ws_bytes, int* nsplit, sel_stream_t stream);
int sel_wgrad_finish_many(const sel_wgrad_job* jobs, int njobs, sel_stream_t stream);
/* Repack fp32 torch weights (kind SEL_PACK_*) into Wp (dtype), and the dgrad
 * form of a packed Wp[N][K][C] -> Wd[C][K][N] with taps reversed (the adjoint is
 * the same primitive with pad' = (K-1)*dil - pad). */
int sel_pack_weight(int kind, const float* w, int cout, int cin, int k, int stride,
                    int dtype, void* wpack, sel_stream_t stream);
int sel_pack_dgrad(const void* wpack, int N, int K, int C, int dtype, void* wd,
                   sel_stream_t stream);
/* Batched form of sel_pack_weight + sel_pack_dgrad for many layers in one launch.
 * `jobs` is a DEVICE array of njobs entries sorted by `offset` (the prefix sum of
 * each job's packed element count); total = sum of the counts.  wdgrad may be NULL. */
typedef struct sel_pack_job {
  const float* w;     /* torch-layout fp32 weight */
  void* wpack;        /* Wp (dtype) */
  void* wdgrad;       /* dgrad form of Wp (dtype) or NULL */
  int64_t offset;
  int32_t kind, cout, cin, k, stride, reserved;
} sel_pack_job;
int sel_pack_many(const sel_pack_job* jobs, int njobs, int64_t total, int dtype, sel_stream_t stream);
/* The same with `jobs` in HOST memory (copied into the kernel arguments, 48
 * jobs per launch; offsets increasing): no device job table to stage.  The
 * product path (sel.convops.PackCache) uses this one. */
int sel_pack_many_host(const sel_pack_job* jobs, int njobs, int64_t total, int dtype, sel_stream_t stream);
/* gwpack (packed fp32) -> torch layout gw (kind as in sel_pack_weight). */
int sel_unpack_wgrad(int kind, const float* gwpack, int cout, int cin, int k, int stride,
                     float* gw, sel_stream_t stream);
/* adjoint of SEL_PAD_REPLICATE (pad 1, K 2): gin[b*T + 0, c] += sum_n gout[b*T + 0, n] * Wp[n][0][c] */
int sel_conv_replicate_fix(const sel_conv_desc* d, int dtype, const void* gout,
                           const void* wpack, void* gin, sel_stream_t stream);
/* dtype casts (activations in/out of the bf16 path) */
int sel_cast(const void* src, int src_dtype, void* dst, int dst_dtype, int64_t n,
             sel_stream_t stream);

/* ---- residual VQ: layers/vq_module.py:61-88 (eval), :119-134 -------------
 * All stages of one row block in one launch (rows are independent):
 *   dist_k = (|r|^2 - (2r).e_k) + |e_k|^2, idx = argmin (lowest index on ties),
 *   q = e_idx, qst = r + (q - r), r <- r - qst, out += qst.
 * x (N, D) fp32; embeds (S, D, K) fp32 (the `embed` buffers stacked);
 * out (N, D); idx (S, N) int64; counts (S, K) int32 (zeroed by the call);
 * sqerr (S) fp64: sum (q - r)^2 per stage. */
size_t sel_rvq_workspace(int64_t N, int S, int K);
int sel_rvq_fwd(const float* x, int64_t N, int D, const float* embeds, int S, int K,
                float* out, int64_t* idx, int32_t* counts, double* sqerr,
                void* ws, size_t ws_bytes, sel_stream_t stream);
/* per-stage loss = sqerr/(N*D)*commitment and perplexity from counts -> loss[S], ppl[S] */
int sel_rvq_finish(const int32_t* counts, const double* sqerr, int64_t N, int D, int S, int K,
                   float commitment, float* loss, float* ppl, sel_stream_t stream);
/* g_x = g_out + g_loss[0]*commitment*2*(x - e0[idx0])/(N*D)  (only stage 0's
 * commitment term reaches x: later residuals have zero Jacobian w.r.t. x, vq_module.py:83,129) */
int sel_rvq_bwd(const float* x, int64_t N, int D, const float* embed0, int K, const int64_t* idx0,
                const float* g_out, const float* g_loss, float commitment, float* g_x,
                sel_stream_t stream);

/* ---- data glue: dataloader/data_utils.py:12-22 (add_noise) ---------------
 * out = (exp(snr/10) * ||noise||_2 / ||speech||_2 * speech + noise) / 2 with
 * BATCH-GLOBAL norms over all n elements (math.exp, not 10^x, as the reference). */
size_t sel_add_noise_workspace(int64_t n);
int sel_add_noise(const float* speech, const float* noise, int64_t n, float snr, float* out,
                  void* ws, size_t ws_bytes, sel_stream_t stream);
/* the same in two halves for data-parallel mixing: per-rank sums2 = {sum s^2, sum n^2}
 * (device doubles, all-reduced by the caller across ranks), then the mix */
int sel_sumsq2(const float* speech, const float* noise, int64_t n, double* sums2, void* ws,
               size_t ws_bytes, sel_stream_t stream);
int sel_mix_noise(const float* speech, const float* noise, int64_t n, const double* sums2, float snr,
                  float* out, sel_stream_t stream);

/* ---- BatchNorm1d (models/autoencoder/modules/projector.py:40-44, model='conv1d_bn';
 * replaces torch.nn.BatchNorm1d.forward / its autograd backward) -------------
 * x, y, gy, gx: (rows, C) fp32 channels-last (rows = B*T).  training: batch
 * statistics (biased variance for the normalisation; running_mean / running_var,
 * when given, updated with `momentum` and the unbiased variance, as torch);
 * otherwise the running statistics.  save_mean / save_invstd (C floats) are
 * written by the forward and read by the backward.  gamma / beta may be null
 * (affine=False); ggamma / gbeta / gx may be null (not wanted).  ws: at least
 * sel_batchnorm_workspace(rows, C) bytes. */
size_t sel_batchnorm_workspace(int64_t rows, int C);
int sel_batchnorm_fwd(const float* x, int64_t rows, int C, const float* gamma, const float* beta, int training,
                      float eps, float momentum, float* running_mean, float* running_var, float* save_mean,
                      float* save_invstd, float* y, void* ws, size_t ws_bytes, sel_stream_t stream);
int sel_batchnorm_bwd(const float* x, const float* gy, int64_t rows, int C, const float* gamma,
                      const float* save_mean, const float* save_invstd, int training, float* gx, float* ggamma,
                      float* gbeta, void* ws, size_t ws_bytes, sel_stream_t stream);

/* ---- optimizer step (trainer/trainerGAN.py:271-281 optimizer.step()) ---- */
/* Adam update (torch.optim.Adam semantics: L2 weight decay, no amsgrad /
 * maximize) of nt fp32 tensors in one launch: per element, g += wd p;
 * m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g g;
 * p -= step_size m / (sqrt(v) / bc2_sqrt + eps), step_size = lr / (1 - b1^t),
 * bc2_sqrt = sqrt(1 - b2^t) (computed by the caller from the step count t). */
typedef struct {
  float* p;
  const float* g;
  float* m;  /* exp_avg */
  float* v;  /* exp_avg_sq */
  int64_t n;
} sel_adam_tensor;
int sel_adam_step_many(const sel_adam_tensor* ts, int nt, double beta1, double beta2, double eps,
                       double weight_decay, double step_size, double bc2_sqrt, sel_stream_t stream);
/* The same update with the step count and learning rate on the device (the
 * capturable form: a HIP-graph replay of a training step stays correct, the
 * role of torch.optim.Adam(capturable=True)): *step += 1, then step_size =
 * lr[0] / (1 - b1^t), bc2_sqrt = sqrt(1 - b2^t) computed in double on the
 * device into consts[0..1] (caller-owned, 2 floats), then the update.  One
 * step count for all nt tensors (one parameter group). */
int sel_adam_step_many_dev(const sel_adam_tensor* ts, int nt, double beta1, double beta2, double eps,
                           double weight_decay, const float* lr, float* step, float* consts,
                           sel_stream_t stream);

/* ---- SNR term of train_denoise.py:140 (torchmetrics 1.2.0 SignalNoiseRatio,
 * zero_mean=False): snr_b = 10 log10((sum t^2 + eps) / (sum (t-p)^2 + eps)) over the
 * last dim, out[0] = mean_b snr_b.  bwd: g_p = g * 20/ln10 * (t-p) / (D_b + eps) / B. */
int sel_snr_fwd(const float* pred, const float* target, int64_t B, int64_t T, double* sums /*2B*/,
                float* out, sel_stream_t stream);
int sel_snr_bwd(const float* pred, const float* target, int64_t B, int64_t T, const double* sums,
                const float* g_out, float* g_pred, sel_stream_t stream);

/* ---- data pipeline: band-limited resampling ----
 * replaces torchaudio.functional.resample(x, orig, new) at dataloader/AudioDataset.py:28-33
 * (defaults: sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99; torchaudio 2.1.1
 * restated).  x (n_wavs, len) fp32 -> y (n_wavs, sel_resample_out_len(len, ...)).
 * The tap table [phases][taps] is caller-owned: fill it on the host with
 * sel_resample_kernel and copy it to the device. */
int sel_resample_plan(int orig_freq, int new_freq, int lowpass_filter_width, float rolloff, int* phases,
                      int* taps);
int64_t sel_resample_out_len(int64_t len, int orig_freq, int new_freq);
int sel_resample_kernel(int orig_freq, int new_freq, int lowpass_filter_width, float rolloff, float* table);
int sel_resample(const float* x, int64_t n_wavs, int64_t len, int orig_freq, int new_freq, int lowpass_filter_width,
                 float rolloff, const float* table, float* y, sel_stream_t stream);

/* ---- waveform shape loss (losses/waveform_loss.py:15-74), one window length per call ----
 * L1(maxpool_w(|y_hat|), maxpool_w(|y|)) over (rows, T) -> out[0]; argidx/dsign
 * (rows * (T / w) each) carry the argmax and sign(diff) to the backward, which
 * ADDS g_out[0] * g_mul * d loss / d y_hat into g_yhat (y is not differentiated). */
size_t sel_shape_loss_workspace(int64_t rows, int64_t T, int win);
int sel_shape_loss_fwd(const float* y_hat, const float* y, int64_t rows, int64_t T, int win, int32_t* argidx,
                       float* dsign, float* out, void* ws, size_t ws_bytes, sel_stream_t stream);
int sel_shape_loss_bwd(const float* y_hat, int64_t rows, int64_t T, int win, const int32_t* argidx,
                       const float* dsign, const float* g_out, float g_mul, float* g_yhat, sel_stream_t stream);

/* ---- HiFi-GAN discriminator (GAN mode) ------------------
 * models/vocoder/HiFiGAN.py:308-395 (Discriminator), models/vocoder/modules/
 * discriminator.py:26-447 (HiFiGANPeriod/Scale discriminators and their multi-
 * versions), losses/adversarial_loss.py:13-124, losses/feat_match_loss.py:13-55.
 *
 * One conv primitive over channels-last rows covers every layer and adjoint:
 *   out[b, j, col(g,o)] = sum_{i<K, r<S, c<Cg} Wp[g][o][i][r][c] * x[b, j+q0+i, r*Cs + g*Cg + c]
 * (input rows outside [0, Tv) read as 0), col(g, o) = (o / Ng)*Ns + g*Ng + o % Ng.
 * Strided convs run on the phase view of their input (S = stride phases of C
 * channels per row, Cs = C), their adjoints with So = stride output phases.
 * Epilogue: + bias[col], then (+ res) * LeakyReLU'(aux) when aux != NULL, then
 * LeakyReLU(slope) when act = 1; rows j in [Tvalid, Tvo) are written as 0. */
typedef struct sel_dconv_desc {
  int32_t B;       /* sequences */
  int32_t Tv;      /* input rows per sequence read (rows >= Tv read as 0) */
  int32_t Tvs;     /* input rows allocated per sequence (>= Tv) */
  int32_t ldx;     /* input row pitch (elements) */
  int32_t Tvo;     /* output rows per sequence (allocated) */
  int32_t Tvalid;  /* computed output rows per sequence */
  int32_t ldo;     /* output row pitch (elements) */
  int32_t K;       /* taps */
  int32_t q0;      /* row offset of tap 0 */
  int32_t S, Cs, Cg; /* reduction: S phases (stride Cs columns) x Cg channels per group */
  int32_t G;       /* groups */
  int32_t So, Ns, Ng; /* outputs: So phases (stride Ns columns) x Ng channels per group */
  int32_t act;     /* 0 none, 1 LeakyReLU */
  float slope;     /* LeakyReLU negative slope (nonlinear_activation_params) */
} sel_dconv_desc;
/* kernel family a sel_dconv_fwd launch of this shape takes (the launcher's own
 * decision, current tune knobs included); writes the kernel's name as rocprofv3
 * lists it (template arguments of the tile) into name[cap] when name != NULL.
 * Returns -1 for an invalid descriptor. */
enum {
  SEL_DPATH_VALU = 0,    /* generic VALU kernel */
  SEL_DPATH_MFMA = 1,    /* matrix-core tile, synchronous stages (grouped layers) */
  SEL_DPATH_SHORT = 2,   /* short reduction (1-channel convs), unstaged */
  SEL_DPATH_PF = 3,      /* matrix-core tile with register prefetch (one group, K <= 8) */
  SEL_DPATH_WS = 4,      /* warp-specialised 256 x 128 kernel, per-sequence tiles */
  SEL_DPATH_WS_FLAT = 5, /* warp-specialised kernel, flat tiles across zero-gapped sequences */
  SEL_DPATH_TINY = 6,    /* narrow outputs (<= 4 columns) */
  SEL_DPATH_GPF = 7,     /* grouped matrix-core tile with register-prefetched stages */
  SEL_DPATH_SHORTX = 8   /* short reduction with the input tile staged in LDS */
};
int sel_dconv_kernel(const sel_dconv_desc* d, int dtype, char* name, size_t cap);
int sel_dconv_fwd(const sel_dconv_desc* d, int dtype, const void* x, const void* wpack, const float* bias,
                  const void* aux, const void* res, void* out, sel_stream_t stream);
/* phase-view tap geometry of a torch conv (kernel Kt, stride, symmetric pad):
 * K = floor((Kt-1-pad)/stride) - q0 + 1 taps from row offset q0 = floor(-pad/stride) */
int sel_dconv_geometry(int Kt, int stride, int pad, int* K, int* q0);
/* torch weight w[N][Cg][Kt] (Conv1d, groups G; or Conv2d (Kt,1)), optionally
 * weight-normed (wg != NULL: w = wg[n] * v / ||v_n||, v = w), into the forward
 * form Wp[g][n][i][r][c] (mode 0) or the adjoint form Wd[g][(r,c)][K-1-i][n] (mode 1). */
int sel_dconv_pack(int mode, const float* w, const float* wg, int N, int Cg, int Kt, int stride, int pad, int G,
                   int dtype, void* out, sel_stream_t stream);
/* Batched sel_dconv_pack: many (layer, mode) packs in one launch per 24 jobs
 * (`jobs` is a HOST array; the same arithmetic per element as sel_dconv_pack).
 * mode 2: the adjoint form as the transpose of a forward form (dtype) at `w`,
 * e.g. one packed by a mode-0 job of the same call (run after all mode 0 / 1 jobs). */
typedef struct sel_dpack_job {
  const float* w;    /* torch weight (or weight_v); mode 2: the packed forward form */
  const float* wg;   /* weight_g or NULL */
  void* out;         /* packed form (dtype) */
  int32_t mode, N, Cg, Kt, stride, pad, G, reserved;
} sel_dpack_job;
int sel_dconv_pack_many(const sel_dpack_job* jobs, int njobs, int dtype, sel_stream_t stream);
/* weight/bias gradient of a forward layer descriptor (So = 1): gw[N][Cg][Kt] fp32
 * in the torch layout, or, with weight norm (v = the weight_v parameter, wg =
 * weight_g): gw = dL/dv and gg[N] = dL/dg; gb[N] = sum of gout when non-NULL. */
size_t sel_dconv_wgrad_workspace(const sel_dconv_desc* d, int dtype);
int sel_dconv_wgrad(const sel_dconv_desc* d, int dtype, const void* gout, const void* x, int N, int Cg, int Kt,
                    int stride, int pad, const float* v, const float* wg, float* gw, float* gg, float* gb, void* ws,
                    size_t ws_bytes, sel_stream_t stream);
/* sel_dconv_wgrad in two phases, so that several layers' final reductions run
 * as one launch: _partials writes the split partials into ws (which must stay
 * allocated, in stream order, until the finish) and describes the reduction
 * in *job; _finish_many runs the reductions of njobs layers (gw / gg / gb as
 * sel_dconv_wgrad writes them). */
typedef struct {
  const float* part;   /* folded split partials (in the layer's ws) */
  const float* bpart;  /* bias partials or NULL */
  const float* v;      /* weight_v or NULL */
  const float* wg;     /* weight_g or NULL */
  float* gw;
  float* gg;
  float* gb;
  int32_t N, Cg, Kt, stride, pad, G, nsplit, bsplit;
} sel_dwgrad_job;
int sel_dconv_wgrad_partials(const sel_dconv_desc* d, int dtype, const void* gout, const void* x, int N, int Cg,
                             int Kt, int stride, int pad, const float* v, const float* wg, float* gw, float* gg,
                             float* gb, void* ws, size_t ws_bytes, sel_dwgrad_job* job, sel_stream_t stream);
int sel_dconv_wgrad_finish_many(const sel_dwgrad_job* jobs, int njobs, sel_stream_t stream);
/* AvgPool1d(kernel, stride, padding, count_include_pad) between MSD scales
 * (discriminator.py:428-447): (B, T) rows of pitch ldx -> (B, To) rows of pitch ldo
 * (positions >= To zero-filled); backward overwrites gx. */
int sel_avgpool1d_fwd(const float* x, int B, int T, int ldx, int kernel, int stride, int pad, int To, int ldo,
                      float* y, sel_stream_t stream);
int sel_avgpool1d_bwd(const float* gy, int B, int T, int ldx, int kernel, int stride, int pad, int To, int ldo,
                      float* gx, sel_stream_t stream);
/* MPD front-end (discriminator.py:120-126): reflect-pad T to a multiple of the
 * period, (B, 1, T/p, p) -> B*p sequences of L = ceil(T/p) rows (pitch Lalloc,
 * rows >= L zero); unfold = the adjoint (folds the reflect pad), overwrites gx. */
int sel_mpd_fold(const float* x, int B, int T, int ldx, int period, int Lalloc, float* y, sel_stream_t stream);
int sel_mpd_unfold(const float* gy, int B, int T, int ldx, int period, int Lalloc, float* gx, sel_stream_t stream);
/* GAN loss reductions over strided views (ndim <= 4, sizes/strides in elements,
 * host arrays): kind 0 = sum|a-b| (feat_match_loss.py:46), 1 = sum (a-target)^2
 * (adversarial_loss.py:57/115/118), 2 = sum min(a-1,0), 3 = sum min(-a-1,0)
 * (hinge, :121/:124), 4 = sum a (generator hinge -mean, :60).  out[0] (+)= scale * sum.  grad (+)= gscale[0] * mult *
 * d(term)/da elementwise (gscale: device scalar, the upstream gradient). */
size_t sel_gan_workspace(void);
int sel_gan_reduce(int kind, int dtype, const void* a, const int64_t* a_size, const int64_t* a_stride,
                   const void* b, const int64_t* b_size, const int64_t* b_stride, int ndim, float target,
                   double scale, int accumulate, float* out, void* ws, size_t ws_bytes, sel_stream_t stream);
int sel_gan_grad(int kind, int dtype, const void* a, const int64_t* a_size, const int64_t* a_stride, const void* b,
                 const int64_t* b_size, const int64_t* b_stride, int ndim, float target, const float* gscale,
                 float mult, void* grad, const int64_t* g_stride, int accumulate, sel_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SEL_H_ */
