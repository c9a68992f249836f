"""Replica sharding: which supervisor replica owns a run.

The reference scales by adding replicas that all process every event
(``/root/reference/.helm/values.yaml:124-125`` "Increase to support higher (1000+)
pod numbers"): N replicas do N times the work and race on every row.  This build
partitions runs over ``sharding.shards`` shards instead; a replica owns a *set* of
shards, fixed (``sharding.mode: static`` → ``{shard-index}``) or held through one
Lease per shard (``mode: lease``, :mod:`..ha.shards`), so a dead replica's shards
fail over one by one to the survivors.

The shard of a run is a function of the Job name (= request id) alone, the one key
every Job, Pod (``batch.kubernetes.io/job-name`` label) and Job Event carries: the
native watch router (``csrc/kube/watch_decoder.cpp`` ``ShardRouter.set_replica``)
drops another replica's lines from the raw bytes, before anything is decoded, so a
replica watching the whole namespace pays only a key scan for the runs it does not
own.  ``SHARD_SEED`` decorrelates replica shards from the worker placement inside a
replica (:data:`.workers._SEED`).
"""
from __future__ import annotations

import time
import zlib
from typing import Dict, FrozenSet, Iterable, Optional, Tuple

SHARD_SEED = 0x5BD1E995


def _fmix32(h: int) -> int:
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    return h ^ (h >> 16)


def shard_of(request_id: str, shards: int) -> int:
    """Replica shard of a run (its Job name); must match the native router.

    CRC32 is affine: for equal-length keys crc32(x, a) ^ crc32(x, b) is a constant, so
    a second CRC seed alone would correlate the replica shard with the worker placement
    (``crc32(x, _SEED) % K``) — with 2 shards and 2 workers every run of a replica would
    land on one worker.  The murmur3 finaliser breaks the linearity."""
    if shards <= 1:
        return 0
    return _fmix32(zlib.crc32(request_id.encode(), SHARD_SEED)) % shards


def shard_selector(label: str, owned: Optional[Iterable[int]], shards: int) -> str:
    """Server-side label selector requirement for the replica's shards of Pods and Jobs
    (``sharding.shard-label``): ``"<label> in (k1,k2,…)"``; ``""`` when off or when the
    replica owns every shard.  Owning none yields a set no run's label can match (a
    lease-mode replica between leases watches nothing)."""
    if not label or shards <= 1 or owned is None:
        return ""
    ks = sorted(int(k) for k in owned)
    if len(ks) == shards:
        return ""
    return f"{label} in ({','.join(str(k) for k in ks) or 'none'})"


def watch_selector(cfg, kind: str, owned: Optional[Iterable[int]] = None) -> str:
    """The server-side label selector of a replica's ``kind`` watch: Nexus runs only
    (``informer-label-selector``) and, with ``sharding.shard-label``, only the replica's
    shards (Pods and Jobs; Events carry neither label)."""
    if kind not in ("Pod", "Job"):
        return ""
    parts = []
    if cfg.informer_label_selector:
        parts.append(f"{cfg.labels.nexus_component_label}={cfg.labels.algorithm_run_value}")
    s = cfg.sharding
    if s.shard_label and s.shards > 1:
        sel = shard_selector(s.shard_label, owned, s.shards)
        if sel:
            parts.append(sel)
    return ",".join(parts)


def watch_field_selector(cfg, kind: str) -> str:
    """The server-side field selector of a replica's ``kind`` watch: on Events
    (``informer-event-noise-selector``), ``reason!=…`` for the start/stop reasons no rule
    reads (:func:`..classify.classifier.event_field_selector`).  The reference watches
    every Event of the namespace (``/root/reference/services/supervisor.go:73-75``)."""
    if kind != "Event" or not getattr(cfg, "informer_event_noise_selector", False):
        return ""
    from ..classify.classifier import event_field_selector

    return event_field_selector(cfg.gpu.gpu_resource_name)


def kube_name(obj) -> str:
    return ((obj or {}).get("metadata") or {}).get("name", "")


class ShardSet:
    """The shards this replica currently owns, with a fencing epoch per shard.

    ``owned`` None means "every shard" (sharding off).  An epoch is bumped whenever the
    shard is lost, so a decision dequeued before the loss never writes after it.

    ``leased`` sets (``sharding.mode: lease``) also carry a per-shard hold deadline
    (``CLOCK_MONOTONIC`` seconds — one clock for every process of the host, so a shard
    worker compares its parent's deadlines directly): a shard whose hold lapsed is not
    owned any more, even before the lease manager's fencing reaches this process."""

    def __init__(self, shards: int = 1, owned: Optional[Iterable[int]] = None, leased: bool = False,
                 clock=time.monotonic):
        self.shards = max(1, int(shards))
        # one shard is "everything" unless it is leased: then the lease is the ownership
        self.owned: Optional[FrozenSet[int]] = (None if owned is None or (self.shards <= 1 and not leased)
                                                else frozenset(owned))
        self.epochs = [0] * self.shards
        self.leased = leased and self.owned is not None
        self.valid_until = [float("-inf") if self.leased else float("inf")] * self.shards
        self.clock = clock

    @classmethod
    def from_config(cls, cfg) -> "ShardSet":
        s = cfg.sharding
        if s.mode == "lease":
            # nothing until a shard lease is won (also with one shard: the lease then is the
            # replica's only ownership, so a replica that never won it writes nothing)
            return cls(max(1, s.shards), (), leased=True)
        if s.shards <= 1:
            return cls(1)
        return cls(s.shards, (s.shard_index,))

    @property
    def enabled(self) -> bool:
        return self.owned is not None

    def of(self, request_id: str) -> int:
        return shard_of(request_id, self.shards)

    def owns(self, request_id: str) -> bool:
        if self.owned is None:
            return True
        k = shard_of(request_id, self.shards)
        return k in self.owned and (not self.leased or self.clock() < self.valid_until[k])

    def set_deadlines(self, until: Dict[int, float]) -> None:
        """Hold deadlines of leased shards (monotonic seconds), from the lease manager."""
        for k, t in until.items():
            k = int(k)
            if 0 <= k < self.shards:
                self.valid_until[k] = float(t)

    def token(self, request_id: str) -> int:
        return self.epochs[shard_of(request_id, self.shards)] if self.owned is not None else 0

    def update(self, owned: Iterable[int]) -> Tuple[FrozenSet[int], FrozenSet[int]]:
        """Replace the owned set; returns (gained, lost) and fences the lost shards."""
        new = frozenset(int(k) for k in owned)
        if any(not 0 <= k < self.shards for k in new):
            raise ValueError(f"shard index out of range [0, {self.shards})")
        old = self.owned if self.owned is not None else frozenset(range(self.shards))
        self.owned = new
        lost = old - new
        for k in lost:
            self.epochs[k] += 1
        return new - old, lost

