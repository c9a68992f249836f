"""Watch-delivery stamps: where an object's change spends its time between the API
server's push and the supervisor's handler, so the open-loop p99 can be split into
transport, hub, feed and dispatch time.

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
(``receive_to_checkpoint``), itself split by :func:`record` at the decision's enqueue and
dequeue.  A failure whose decision waited (a ``pods/log`` tail, node-agent evidence) keeps
the receive time and delivery stamps of the update that carried it.
"""
from __future__ import annotations

from typing import Any, Dict, List, Tuple

CURRENT: Dict[str, Tuple[float, float, float]] = {}


def record(stamps: Dict[str, Any], dl: Tuple[float, float, float]) -> List[float]:
    """``[hub, feed, dec, classify, queue, receive→ack]`` of one decision: the delivery
    stamps (monotonic), then seconds from the handler's receive to the pipeline enqueue
    (classification, including any wait for a log tail), enqueue → dequeue (the keyed
    queue), and receive → checkpoint ack."""
    rcv = stamps["receive"]
    enq = stamps.get("enqueue", rcv)
    deq = stamps.get("dequeue", enq)
    return [dl[0], dl[1], dl[2], enq - rcv, deq - enq, stamps["ack"] - rcv]
