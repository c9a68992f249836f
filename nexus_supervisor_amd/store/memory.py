"""In-process checkpoint store (``cql-store-type: memory``): tests, dry runs, benches
that isolate the supervisor from CQL."""
from __future__ import annotations

import asyncio
import datetime as _dt
from typing import Dict, Iterable, Optional, Tuple

from ..models.checkpoint import CheckpointedRequest
from .base import CheckpointStore, StoreError


class MemoryStore(CheckpointStore):
    def __init__(self, rows: Iterable[CheckpointedRequest] = (), latency: float = 0.0):
        self.rows: Dict[Tuple[str, str], CheckpointedRequest] = {r.key: r.deep_copy() for r in rows}
        self.latency = latency
        self.reads = 0
        self.writes = 0
        self.fail_next_reads = 0
        self.fail_next_writes = 0
        self.write_log: list = []  # (key, stage) of every applied write (tests: exactly-once checks)

    async def _io(self):
        if self.latency:
            await asyncio.sleep(self.latency)

    async def read_checkpoint(self, algorithm: str, request_id: str) -> Optional[CheckpointedRequest]:
        await self._io()
        self.reads += 1
        if self.fail_next_reads:
            self.fail_next_reads -= 1
            raise StoreError("injected read failure")
        r = self.rows.get((algorithm, request_id))
        return r.deep_copy() if r else None

    async def upsert_checkpoint(self, checkpoint: CheckpointedRequest) -> None:
        await self._io()
        self.writes += 1
        if self.fail_next_writes:
            self.fail_next_writes -= 1
            raise StoreError("injected write failure")
        self.rows[checkpoint.key] = checkpoint.deep_copy()
        self.write_log.append((checkpoint.key, checkpoint.lifecycle_stage))

    async def update_status(self, algorithm, request_id, lifecycle_stage, failure_cause, failure_details,
                            last_modified: _dt.datetime, only_if_stages=None, set_failure=True) -> bool:
        await self._io()
        self.writes += 1
        if self.fail_next_writes:
            self.fail_next_writes -= 1
            raise StoreError("injected write failure")
        key = (algorithm, request_id)
        row = self.rows.get(key)
        if only_if_stages is not None:
            if row is None or row.lifecycle_stage not in set(only_if_stages):
                return False
        if row is None:  # CQL UPDATE is an upsert
            row = CheckpointedRequest(algorithm=algorithm, id=request_id)
        row = row.deep_copy()
        row.lifecycle_stage = lifecycle_stage
        if set_failure:
            row.algorithm_failure_cause = failure_cause
            row.algorithm_failure_details = failure_details
        row.last_modified = last_modified
        self.rows[key] = row
        self.write_log.append((key, lifecycle_stage))
        return True

    async def cas_update(self, algorithm, request_id, lifecycle_stage, failure_cause, failure_details,
                         last_modified: _dt.datetime, only_if_stages, set_failure=True) -> Tuple[bool, Optional[str]]:
        """Atomic in one step (no await between the check and the write), like the LWT."""
        await self._io()
        self.reads += 1
        self.writes += 1
        if self.fail_next_writes:
            self.fail_next_writes -= 1
            raise StoreError("injected write failure")
        key = (algorithm, request_id)
        row = self.rows.get(key)
        if row is None:
            return False, None
        if row.lifecycle_stage not in set(only_if_stages):
            return False, row.lifecycle_stage
        row = row.deep_copy()
        row.lifecycle_stage = lifecycle_stage
        if set_failure:
            row.algorithm_failure_cause = failure_cause
            row.algorithm_failure_details = failure_details
        row.last_modified = last_modified
        self.rows[key] = row
        self.write_log.append((key, lifecycle_stage))
        return True, None

    def get(self, algorithm: str, request_id: str) -> Optional[CheckpointedRequest]:
        return self.rows.get((algorithm, request_id))
