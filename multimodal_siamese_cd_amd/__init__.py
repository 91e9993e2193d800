"""MI355X-native (gfx950) Siamese change-detection U-Net training path.

Drop-in for SebastianHafner/multimodal_siamese_cd's `utils.networks` / `utils.loss_functions` /
`utils.experiment_manager` surface; the compute runs in libscd.so (hand-written HIP, see include/scd.h).
"""
__version__ = "0.1.0"
