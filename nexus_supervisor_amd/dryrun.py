"""Shadow mode (``dry-run: true``): the supervisor watches, classifies, attributes and
decides exactly as in production, and reads the checkpoint rows it needs, but never
writes a row or deletes a Job.  Each would-be action is logged at INFO with everything
the write would have carried, and counted (``dry_run_writes{stage}``,
``dry_run_deletes``).

The point is migration: the reference acts on every event it sees and has no such mode
(``/root/reference/services/supervisor.go:261-374`` deletes and upserts unconditionally),
so the only way to compare it with a replacement used to be to let both act.  In shadow
mode this supervisor runs next to the reference on production traffic and its decision
log can be diffed against the rows the reference writes — including the classes the
reference cannot produce (HBM-OOM with its GPU, evictions, image pulls) — before it is
given the checkpoint table.

Both wrappers sit at the composition root (:class:`..app.Application`), so the
single-process replica and every shard worker of a process-per-core replica behave the
same; everything that is not a write is delegated unchanged (reads, ``pods/log`` tails,
connection management).
"""
from __future__ import annotations

import datetime as _dt
from typing import Any, Iterable, Optional, Tuple

from .models.checkpoint import CheckpointedRequest
from .store.base import CheckpointStore


class DryRunStore(CheckpointStore):
    """Reads go to ``inner``; writes are logged and answered as the store would have
    (a conditional write is "applied" iff the row's current stage satisfies the guard)."""

    def __init__(self, inner: CheckpointStore, log, metrics):
        self.inner = inner
        self.log = log
        self.metrics = metrics
        self.writes = 0

    def __getattr__(self, name: str) -> Any:
        return getattr(self.inner, name)

    async def read_checkpoint(self, algorithm: str, request_id: str) -> Optional[CheckpointedRequest]:
        return await self.inner.read_checkpoint(algorithm, request_id)

    async def read_status(self, algorithm: str, request_id: str) -> Optional[CheckpointedRequest]:
        return await self.inner.read_status(algorithm, request_id)

    async def connect(self) -> None:
        await self.inner.connect()

    async def close(self) -> None:
        await self.inner.close()

    def _would_write(self, algorithm: str, request_id: str, stage: str, cause: Optional[str],
                     details: Optional[str], current: Optional[str], how: str) -> None:
        self.writes += 1
        self.metrics.inc("dry_run_writes", labels={"stage": stage})
        self.log.info("dry run: checkpoint not written", requestId=request_id, algorithm=algorithm, stage=stage,
                      currentStage=current, write=how, algorithmFailureCause=cause,
                      algorithmFailureDetails=details)

    async def upsert_checkpoint(self, checkpoint: CheckpointedRequest) -> None:
        self._would_write(checkpoint.algorithm, checkpoint.id, checkpoint.lifecycle_stage,
                          checkpoint.algorithm_failure_cause, checkpoint.algorithm_failure_details, None, "upsert")

    async def update_status(self, algorithm: str, request_id: str, lifecycle_stage: str, failure_cause: Optional[str],
                            failure_details: Optional[str], last_modified: _dt.datetime,
                            only_if_stages: Optional[Iterable[str]] = None, set_failure: bool = True) -> bool:
        current = None
        if only_if_stages is not None:
            cp = await self.inner.read_status(algorithm, request_id)
            current = cp.lifecycle_stage if cp is not None else None
            if current not in tuple(only_if_stages):
                return False  # the conditional write would not have applied
        self._would_write(algorithm, request_id, lifecycle_stage, failure_cause if set_failure else None,
                          failure_details if set_failure else None, current,
                          "conditional" if only_if_stages is not None else "update")
        return True

    async def cas_update(self, algorithm: str, request_id: str, lifecycle_stage: str, failure_cause: Optional[str],
                         failure_details: Optional[str], last_modified: _dt.datetime, only_if_stages: Iterable[str],
                         set_failure: bool = True) -> Tuple[bool, Optional[str]]:
        cp = await self.inner.read_status(algorithm, request_id)
        if cp is None:
            return False, None
        if cp.lifecycle_stage not in tuple(only_if_stages):
            return False, cp.lifecycle_stage
        self._would_write(algorithm, request_id, lifecycle_stage, failure_cause if set_failure else None,
                          failure_details if set_failure else None, cp.lifecycle_stage, "fused")
        return True, None


class DryRunJobs:
    """Job client whose DELETE is logged instead of sent; everything else (``pods/log``
    reads, the API client's lifecycle) is delegated."""

    def __init__(self, inner, log, metrics):
        self.inner = inner
        self.log = log
        self.metrics = metrics
        self.deletes = 0

    def __getattr__(self, name: str) -> Any:
        if name == "delete_job_nowait":
            raise AttributeError(name)  # the supervisor then takes the coroutine path below
        return getattr(self.inner, name)

    async def delete_job(self, namespace: str, name: str, propagation_policy: str = "Background") -> None:
        self.deletes += 1
        self.metrics.inc("dry_run_deletes")
        self.log.info("dry run: Job not deleted", requestId=name, namespace=namespace,
                      propagationPolicy=propagation_policy)
