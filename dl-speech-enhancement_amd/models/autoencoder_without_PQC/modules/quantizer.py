from models.autoencoder.modules.quantizer import *  # noqa: F401,F403
