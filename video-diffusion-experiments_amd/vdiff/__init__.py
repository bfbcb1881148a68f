"""vdiff — MI355X-native video-diffusion denoising step (AnimateDiff UNetMotionModel + DDIM / Euler).

Host mirror of the reference's call surface (diffusers UNetMotionModel /
DDIMScheduler / AnimateDiffPipeline as used by tanm-ast/video-diffusion-
experiments) over hand-written gfx950 HIP kernels in libvdiff_hip.so.
"""
from .config import FULL, TINY, get_config  # noqa: F401
from .models import UNetMotionModel, UNetMotionOutput  # noqa: F401
from .models.dit import DiT3DModel, DiTDenoiseLoop, DiTOutput  # noqa: F401
from .models.vae import AutoencoderKL, DecoderOutput  # noqa: F401
from .pretrained import MotionAdapter  # noqa: F401
from .pipeline import AnimateDiffPipeline, AnimateDiffPipelineOutput, DenoiseLoop  # noqa: F401
from .sched import (DDIMScheduler, DDIMSchedulerOutput, EulerDiscreteScheduler,  # noqa: F401
                    EulerDiscreteSchedulerOutput)
from .weights import init_synthetic_, load_diffusers_state_dict  # noqa: F401
