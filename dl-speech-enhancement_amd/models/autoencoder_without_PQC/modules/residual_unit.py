from models.autoencoder.modules.residual_unit import *  # noqa: F401,F403
