"""gossipprotocol_amd -- MI355X-native synchronous gossip / push-sum simulator.

Drop-in for the hot path of sharwarimarathe/GossipProtocol
(`dotnet run num_nodes topology algorithm`, Program.fs:31-283): the per-round
message delivery of gossip and push-sum on line / full / 3D / Imp3D
topologies plus the convergence check, as HIP kernels for gfx950 behind the
C-ABI in include/gossip_hip.h.  See DESIGN.md.
"""
from .sim import ALGORITHMS, TOPOLOGIES, Simulation, parse_algorithm, parse_topology, resolve, run  # noqa: F401

__version__ = "1.0.0"
