from .ddim import DDIMScheduler, DDIMSchedulerOutput  # noqa: F401
