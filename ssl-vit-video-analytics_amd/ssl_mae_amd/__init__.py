"""ssl_mae_amd — MI355X-native (gfx950) video-MAE pretraining hot path of
lzc452/SSL-VIT-VIDEO-ANALYTICS: HIP kernels behind a C ABI (libsslmae.so) with a
host mirror of the reference's module API (tiny_vit_21m_variant, TinyVideoMAE,
get_tube_mask, patchify, train_one_epoch)."""
__version__ = "0.1.0"
