from .frame_shard import FrameShard, block_transpose_reference, rev3_reference  # noqa: F401
from .layout import CfgShard, NodeLayout  # noqa: F401
