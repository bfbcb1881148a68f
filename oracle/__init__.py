"""ORACLE — CPU restatement of the reference's denoising step (test infrastructure).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / CPU baseline.  The product package
(video-diffusion-experiments_amd/vdiff) never imports it and has no CPU
fallback.  Parity vs diffusers is UNPINNED (diffusers is absent, no reference
tensors exist); the module tree is pinned by the reference's structural
known-answers.  See DESIGN.md §Oracle.
"""
from . import ddim_ref, unet_ref  # noqa: F401
