"""nexus_supervisor_amd — a job supervisor for Kubernetes clusters of AMD MI355X GPUs.

Same capabilities, config surface and ``nexus.checkpoints`` schema as
SneaksAndData/nexus-supervisor (reference snapshot at ``/root/reference``),
re-designed: asyncio control plane, native C++ CQL wire codec, amd-smi GPU
attribution (HBM-OOM vs host-OOM on 288 GB HBM3E), RCCL/xGMI rank topology in
the trace row, keyed work pipeline, leader election and pprof-format profiling.
"""
from .buildmeta import APP_VERSION as __version__, BUILD_NUMBER as __build__  # noqa: E402,F401

import os as _os

# Sanitizer runs (tests/test_sanitizers.py): resolve the native extensions from an
# instrumented build directory first.
if _os.environ.get("NEXUS_NATIVE_DIR"):
    __path__.insert(0, _os.environ["NEXUS_NATIVE_DIR"])  # type: ignore[name-defined]

# hot-path modules as C extensions when built from the sources on disk (compiled.py)
from . import compiled as _compiled  # noqa: E402

_compiled.install()
