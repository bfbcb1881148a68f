from .unet_motion import UNetMotionModel, UNetMotionOutput  # noqa: F401
