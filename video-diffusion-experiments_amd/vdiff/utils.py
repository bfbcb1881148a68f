"""diffusers.utils stand-ins the reference's sampling scripts import
(experiments/05_grid_search_ablation.py:28 `from diffusers.utils import export_to_gif`;
diffusers.utils.torch_utils.randn_tensor, which AnimateDiffPipeline.prepare_latents calls)."""
from .pipeline import export_to_gif, numpy_to_pil, randn_tensor  # noqa: F401
