"""gossip_hip — MI355X-native gossip-round engine (Python side of include/gossip.h).

The compute path is libgossip_hip.so (hand-written HIP kernels for gfx950);
this package only binds it (ctypes) and orchestrates sharded rounds over
torch.distributed.  See DESIGN.md.
"""
from ._abi import (FLAG_AE_DIRECT_SCAN, FLAG_DENSE, FLAG_DIRECT, FLAG_HASH, FLAG_SHARD_DIRECT, FLAG_TIMING, MODE_FLOOD, MODE_PULL, MODE_PUSH, MODE_PUSHPULL, MODES,
                   Config, RoundStats)
from .engine import (AbiEngine, Engine, GossipError, Group, LIB_PATH, StepResult, comm_unique_id, load_library,
                     loss_threshold, make_config, peer)
from .maelstrom import Cluster, grid_topology, line_topology, total_topology, tree_topology

__all__ = [
    "AbiEngine", "Engine", "GossipError", "Group", "comm_unique_id", "StepResult", "Config", "RoundStats", "MODES", "MODE_FLOOD",
    "MODE_PUSH", "MODE_PULL", "MODE_PUSHPULL", "FLAG_AE_DIRECT_SCAN", "FLAG_SHARD_DIRECT", "FLAG_DENSE", "FLAG_DIRECT", "FLAG_HASH", "FLAG_TIMING", "LIB_PATH", "load_library",
    "make_config", "loss_threshold", "peer", "Cluster", "grid_topology", "line_topology", "total_topology", "tree_topology",
]
