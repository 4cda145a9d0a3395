"""Operator-level entry points (reference core/operators/): HIP replacements of the CuPy kernels
and the plugin-hook registry, all calling libvcap_hip.so through its C ABI."""
