"""cilium_amd — MI355X-native batched flow classification for Cilium's L3/L4
datapath decision (ipcache LPM identity, XDP CIDR prefilter, per-endpoint
policy-map verdict), behind a C ABI (include/cgpu.h).

Importing the package loads nothing; :mod:`cilium_amd.engine` loads
``libcgpu.so`` and raises if it is missing (no CPU fallback exists).
"""

__all__ = ["layouts", "engine", "build", "synth"]
