from .ddim import DDIMScheduler, DDIMSchedulerOutput  # noqa: F401
from .euler import EulerDiscreteScheduler, EulerDiscreteSchedulerOutput  # noqa: F401
