"""Checkpoint store protocol.

nexus-core ``request.CqlStore`` exposes ``ReadCheckpoint(algorithm, id)`` and
``UpsertCheckpoint(*CheckpointedRequest)`` (call sites
``/root/reference/services/supervisor.go:264,301,328,353,364``).  This build
keeps both and adds :meth:`CheckpointStore.update_status`, an owned-columns
write (``UPDATE … SET lifecycle_stage, algorithm_failure_cause,
algorithm_failure_details, last_modified``) that cannot clobber columns other
Nexus components own, optionally conditional on the row still
being unfinished (lightweight transaction).
"""
from __future__ import annotations

import datetime as _dt
from typing import Iterable, Optional, Tuple

from ..models.checkpoint import CheckpointedRequest


class StoreError(Exception):
    """Transient or permanent store failure (the pipeline retries it).  ``availability``:
    the error says the *store* is unreachable or overloaded (what the circuit breaker
    counts), not that one request was refused (an invalid query, one partition's write
    timeout, LWT contention)."""

    availability = True


def is_availability_error(exc: BaseException) -> bool:
    return isinstance(exc, StoreError) and bool(getattr(exc, "availability", True))


class NotSent(StoreError):
    """The request never reached any replica (no live host / connection): the write
    certainly did not land."""


class CheckpointStore:
    async def read_checkpoint(self, algorithm: str, request_id: str) -> Optional[CheckpointedRequest]:
        raise NotImplementedError

    async def read_status(self, algorithm: str, request_id: str) -> Optional[CheckpointedRequest]:
        """The row's key and ``lifecycle_stage`` only — all the owned-columns write path
        needs (``is_finished`` and the CAS guard).  Stores that can project the read
        (CQL: ``SELECT lifecycle_stage``) override this; the default reads the full row."""
        return await self.read_checkpoint(algorithm, request_id)

    async def upsert_checkpoint(self, checkpoint: CheckpointedRequest) -> None:
        raise NotImplementedError

    async def update_status(
        self,
        algorithm: str,
        request_id: str,
        lifecycle_stage: str,
        failure_cause: Optional[str],
        failure_details: Optional[str],
        last_modified: _dt.datetime,
        only_if_stages: Optional[Iterable[str]] = None,
        set_failure: bool = True,
    ) -> bool:
        """Write the owned columns. With ``only_if_stages`` the write is a CAS
        (``IF lifecycle_stage IN (...)``); returns whether it was applied."""
        raise NotImplementedError

    async def cas_update(
        self,
        algorithm: str,
        request_id: str,
        lifecycle_stage: str,
        failure_cause: Optional[str],
        failure_details: Optional[str],
        last_modified: _dt.datetime,
        only_if_stages: Iterable[str],
        set_failure: bool = True,
    ) -> Tuple[bool, Optional[str]]:
        """Fused read-modify-write (``compat.fused-write``): the conditional write alone
        decides, so the actuator needs no prior read.  Returns ``(applied, stage)`` where
        ``stage`` is the row's current stage when the condition failed (None: no row).
        Stores that cannot do it atomically fall back to read + conditional write."""
        only_if_stages = tuple(only_if_stages)
        cp = await self.read_status(algorithm, request_id)
        if cp is None:
            return False, None
        if cp.lifecycle_stage not in only_if_stages:
            return False, cp.lifecycle_stage
        applied = await self.update_status(algorithm, request_id, lifecycle_stage, failure_cause, failure_details,
                                           last_modified, only_if_stages=only_if_stages, set_failure=set_failure)
        if applied:
            return True, None
        cp = await self.read_status(algorithm, request_id)
        return False, cp.lifecycle_stage if cp is not None else None

    async def connect(self) -> None:
        return None

    async def close(self) -> None:
        return None
