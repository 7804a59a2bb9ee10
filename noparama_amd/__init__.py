"""noparama_amd -- MI355X-native Neal Algorithm 8 Gibbs sweep for Dirichlet-process mixtures of
multivariate normals, behind the sampler plug-in API of mrquincle/noparama.

The product is the HIP/C library noparama_amd/lib/libnp8.so (C ABI: include/np8.h); this package
is its ctypes binding plus data helpers for tests and the benchmark.
"""
from .np8 import (NP8_REQ_MAX, JainNealAlgorithm, NealAlgorithm8, NP8Error, TriadicAlgorithm,  # noqa: F401
                  comm_unique_id, header_symbols, lib, membertrix)

__all__ = ["NealAlgorithm8", "JainNealAlgorithm", "TriadicAlgorithm", "NP8Error", "membertrix", "lib", "header_symbols",
           "comm_unique_id", "NP8_REQ_MAX"]
