"""Hot-path hyper-parameters of the reference configs (no reference YAML is
shipped; these are the keys the training step reads).

* SYMAD_24MEL — config/denoise/symAD_24Mel.yaml (train_denoise.py's config).
* SYMAD_VCTK_48K_GAN — BASELINE config C5 (GAN mode at 48 kHz), from
  config/denoise/symAD_vctk_48000_hop300.yaml.
* SYMAD_LIBRITTS_24K_DENOISE — BASELINE config C4 names
  config/denoise/symAD_libritts_24000_hop300, which does not exist in the
  reference.  Derived from config/autoencoder/symAD_libritts_24000_hop300.yaml
  exactly as the shipped 48 kHz pair differs: train_mode denoise,
  mel win_lengths [null] (== n_fft 2048), batch_length 24000 (1 s).
"""
import copy

GENERATOR = dict(input_channels=1, output_channels=1, encode_channels=32, decode_channels=32, code_dim=64,
                 codebook_num=8, codebook_size=1024, bias=True, enc_ratios=[2, 4, 8, 16],
                 dec_ratios=[16, 8, 4, 2], enc_strides=[3, 4, 5, 5], dec_strides=[5, 5, 4, 3], mode="causal",
                 codec="audiodec", projector="conv1d", quantier="residual_vq")

STFT = dict(fft_sizes=[1024, 2048, 512], hop_sizes=[120, 240, 50], win_lengths=[600, 1200, 240],
            window="hann_window")

# HiFi-GAN MSD + MPD discriminator (config/denoise/symAD_24Mel.yaml:48-82; the
# vctk 48 kHz config :49-82 is identical)
DISCRIMINATOR = dict(
    scales=3, scale_downsample_pooling="AvgPool1d",
    scale_downsample_pooling_params=dict(kernel_size=4, stride=2, padding=2),
    scale_discriminator_params=dict(in_channels=1, out_channels=1, kernel_sizes=[15, 41, 5, 3], channels=128,
                                    max_downsample_channels=1024, max_groups=16, bias=True,
                                    downsample_scales=[4, 4, 4, 4, 1], nonlinear_activation="LeakyReLU",
                                    nonlinear_activation_params=dict(negative_slope=0.1)),
    follow_official_norm=True, periods=[2, 3, 5, 7, 11],
    period_discriminator_params=dict(in_channels=1, out_channels=1, kernel_sizes=[5, 3], channels=32,
                                     downsample_scales=[3, 3, 3, 3, 1], max_downsample_channels=1024, bias=True,
                                     nonlinear_activation="LeakyReLU",
                                     nonlinear_activation_params=dict(negative_slope=0.1),
                                     use_weight_norm=True, use_spectral_norm=False))

ADV = dict(generator_adv_loss_params=dict(average_by_discriminators=False),
           discriminator_adv_loss_params=dict(average_by_discriminators=False),
           use_feat_match_loss=True,
           feat_match_loss_params=dict(average_by_discriminators=False, average_by_layers=False,
                                       include_final_outputs=False))

SYMAD_LIBRITTS_24K_DENOISE = dict(
    sampling_rate=24000, train_mode="denoise", initial="",
    generator_params=GENERATOR,
    use_mel_loss=True,
    mel_loss_params=dict(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None], window="hann_window",
                         num_mels=80, fmin=0, fmax=12000, log_base=None),
    use_stft_loss=False, stft_loss_params=STFT, use_shape_loss=False,
    lambda_adv=1.0, lambda_feat_match=2.0, lambda_vq_loss=1.0, lambda_mel_loss=45.0, lambda_stft_loss=45.0,
    lambda_shape_loss=45.0,
    batch_size=16, batch_length=24000,
    generator_optimizer_type="Adam", generator_optimizer_params=dict(lr=1.0e-4, betas=[0.5, 0.9], weight_decay=0.0),
    generator_scheduler_type="StepLR", generator_scheduler_params=dict(step_size=200000, gamma=1.0),
    generator_grad_norm=-1,
    train_max_steps=200000, save_interval_steps=100000, eval_interval_steps=1000, log_interval_steps=100,
)

SYMAD_24MEL = dict(
    sample_rate=24000, initial_model="", step=0, experiment_name="24Mel", epochs=500,
    epoch_to_enable_discriminator=100, noise_dropout_rate=0.0, noise_dropout_rate_decay=0.05,
    epoch_to_enable_noise_dropout_decay=1000, seed=93, lambda_snr_loss=0.0,
    generator_params=GENERATOR,
    use_mel_loss=True,
    mel_loss_params=dict(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None], window="hann_window",
                         num_mels=80, fmin=0, fmax=24000, log_base=None),
    use_stft_loss=False, stft_loss_params=STFT, use_shape_loss=False,
    lambda_adv=1.0, lambda_feat_match=1000.0, lambda_vq_loss=1.0, lambda_mel_loss=45.0, lambda_stft_loss=45.0,
    lambda_shape_loss=45.0,
    batch_size=8, batch_length=96000,
    generator_optimizer_type="Adam", generator_optimizer_params=dict(lr=5.0e-5, weight_decay=1.0e-6),
    generator_scheduler_type="StepLR", generator_scheduler_params=dict(step_size=200000, gamma=1.0),
    generator_grad_norm=1,
    discriminator_params=DISCRIMINATOR, **ADV,
    discriminator_optimizer_type="Adam", discriminator_optimizer_params=dict(lr=2.0e-4, weight_decay=1.0e-6),
    discriminator_scheduler_type="MultiStepLR",
    discriminator_scheduler_params=dict(gamma=0.5, milestones=[200000, 400000, 600000, 800000]),
    discriminator_grad_norm=1,
)

# BASELINE config C5 (GAN mode, 48 kHz hop 300): config/denoise/symAD_vctk_48000_hop300.yaml's
# generator / discriminator / mel / adversarial / optimizer settings (:30-176) in the
# train_denoise.py key set (the yaml is an AudioDec trainer config and lacks the
# script's schedule keys), discriminator on from the first epoch, 1 s clips (48000).
SYMAD_VCTK_48K_GAN = dict(
    sample_rate=48000, initial_model="", step=0, experiment_name="vctk48-GAN", epochs=500,
    epoch_to_enable_discriminator=0, noise_dropout_rate=0.0, noise_dropout_rate_decay=0.0,
    epoch_to_enable_noise_dropout_decay=1000, seed=93, lambda_snr_loss=0.0,
    generator_params=GENERATOR, discriminator_params=DISCRIMINATOR, **ADV,
    use_mel_loss=True,
    mel_loss_params=dict(fs=48000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None], window="hann_window",
                         num_mels=80, fmin=0, fmax=24000, log_base=None),
    use_stft_loss=False, stft_loss_params=STFT, use_shape_loss=False,
    lambda_adv=1.0, lambda_feat_match=2.0, lambda_vq_loss=1.0, lambda_mel_loss=45.0, lambda_stft_loss=45.0,
    lambda_shape_loss=45.0,
    batch_size=16, batch_length=48000,
    generator_optimizer_type="Adam", generator_optimizer_params=dict(lr=1.0e-4, betas=[0.5, 0.9], weight_decay=0.0),
    generator_scheduler_type="StepLR", generator_scheduler_params=dict(step_size=200000, gamma=1.0),
    generator_grad_norm=-1,
    discriminator_optimizer_type="Adam",
    discriminator_optimizer_params=dict(lr=2.0e-4, betas=[0.5, 0.9], weight_decay=0.0),
    discriminator_scheduler_type="MultiStepLR",
    discriminator_scheduler_params=dict(gamma=0.5, milestones=[200000, 400000, 600000, 800000]),
    discriminator_grad_norm=-1,
)

# noise-dropout continuations of 24Mel (config/denoise/symAD_24MelNDO{,SNR}.yaml, symAD_custom.yaml)
_NDO = dict(noise_dropout_rate=0.8, noise_dropout_rate_decay=0.1, epoch_to_enable_noise_dropout_decay=1,
            experiment_name="24Mel-NDR08-NDRD01-Cont.")
SYMAD_24MEL_NDO = dict(SYMAD_24MEL, **_NDO, initial_model="24kHz-NDR08-NDRD01-SISDRcheckpoint-30701.pkl", step=30701)
SYMAD_24MEL_NDOSNR = dict(SYMAD_24MEL, **_NDO, initial_model="24kHz-NDR08-NDRD01-SNRcheckpoint-55830.pkl",
                          step=55830, lambda_snr_loss=45.0)
SYMAD_CUSTOM = dict(SYMAD_24MEL, **_NDO, sample_rate=48000, step=55830, batch_size=16)

CONFIGS = {"symAD_libritts_24000_hop300": SYMAD_LIBRITTS_24K_DENOISE, "symAD_24Mel": SYMAD_24MEL,
           "symAD_24MelNDO": SYMAD_24MEL_NDO, "symAD_24MelNDOSNR": SYMAD_24MEL_NDOSNR,
           "symAD_custom": SYMAD_CUSTOM, "symAD_vctk_48000_hop300": SYMAD_VCTK_48K_GAN}


def get(name):
    return copy.deepcopy(CONFIGS[name])
