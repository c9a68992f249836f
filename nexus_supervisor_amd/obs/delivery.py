"""Watch-delivery stamps: where an object's change spends its time between the API
server's push and the supervisor's handler (~1.8 ms of the open-loop
p99 sat there, unexplained).

The transport stamps each batch it hands to an informer (CLOCK_MONOTONIC, shared by every
process on the host):

* ``hub``  — the replica's watch hub read the chunk from the API server (parent process);
  the hub-less single-process path stamps its own watch chunk here;
* ``feed`` — the shard worker read the hub's frame off its data socket;
* ``dec``  — the worker's native decoder turned the batch into objects (queue wait +
  decode done).

:data:`CURRENT` holds the stamps of the batch each kind's informer is dispatching right now
(one informer loop per kind, batches dispatched synchronously), so a handler reads them
with one dict lookup; the supervisor copies them into a decision's stamps
(``observability.stage-timestamps``).  Stages: push → hub (simulator / apiserver send +
TCP + the hub's read), hub → feed (routing + the hub → worker frame), feed → dec (worker
queue + decode), dec → handler (informer dispatch), handler → checkpoint ack
(``receive_to_checkpoint``).
"""
from __future__ import annotations

from typing import Dict, Tuple

CURRENT: Dict[str, Tuple[float, float, float]] = {}
