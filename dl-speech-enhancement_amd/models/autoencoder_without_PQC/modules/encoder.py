from models.autoencoder.modules.encoder import *  # noqa: F401,F403
