"""Child-process helpers for the harness servers (CQL server, apiserver simulator,
benchmark cluster process)."""
from __future__ import annotations

import signal


def die_with_parent(sig: int = signal.SIGTERM):
    """``preexec_fn`` for :class:`subprocess.Popen`: the child gets ``sig`` when the thread
    that started it exits (``PR_SET_PDEATHSIG``), so a bench rank killed by its time limit
    does not leave its servers running (they are started in their own session, out of the
    reach of a group kill)."""
    def fn() -> None:
        try:
            import ctypes

            ctypes.CDLL(None, use_errno=True).prctl(1, int(sig))  # PR_SET_PDEATHSIG
        except Exception:  # noqa: BLE001 - best effort (non-Linux)
            pass

    return fn
