from .frame_shard import FrameShard, block_transpose_reference  # noqa: F401
