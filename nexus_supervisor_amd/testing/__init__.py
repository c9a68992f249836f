"""Test/bench infrastructure shipped with the package: parity fixtures, in-process fakes
that speak the real wire protocols (kube-apiserver REST/watch, CQL v4), a fake
amd-smi backend, and synthetic workload generators."""
