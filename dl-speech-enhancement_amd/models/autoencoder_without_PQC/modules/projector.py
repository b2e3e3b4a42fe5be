from models.autoencoder.modules.projector import *  # noqa: F401,F403
