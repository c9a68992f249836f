"""``python -m nexus_supervisor_amd shadow-report LOG [LOG ...]``: how a shadow run
(``dry-run: true``, :mod:`.dryrun`) agrees with the checkpoint rows the acting supervisor
— the reference, during a migration — actually wrote.

Input: the shadow supervisor's JSON log lines (``kubectl logs …``); every
``dry run: checkpoint not written`` line is a decision it would have written.  For each
run (its last such line) the row is read from the store configured as for the supervisor
(``cql-store-type`` and the ``*-cql-store`` section), and the report counts:

* ``agree`` — the store holds the stage the shadow would have written;
* ``differ`` — the store holds another stage (listed with the shadow's failure class:
  a run the reference marked DEADLINE_EXCEEDED that the shadow calls an HBM-OOM shows up
  here as ``hbm-oom``);
* ``unfinished`` — the row is still unfinished (the acting supervisor did not act, or
  has not yet: re-run the report later);
* ``missing`` — no such row.

The reference itself has no way to compare two supervisors (it acts on every decision,
``/root/reference/services/supervisor.go:261-374``).
"""
from __future__ import annotations

import asyncio
import json
import sys
from typing import Any, Dict, Iterable, List, Tuple

from .models import checkpoint as _cp

DRY_RUN_MSG = "dry run: checkpoint not written"


def parse_shadow_log(lines: Iterable[str]) -> Dict[Tuple[str, str], Dict[str, Any]]:
    """(algorithm, request id) → the shadow's last would-be write for that run."""
    out: Dict[Tuple[str, str], Dict[str, Any]] = {}
    for line in lines:
        line = line.strip()
        if not line.startswith("{") or DRY_RUN_MSG not in line:
            continue
        try:
            doc = json.loads(line)
        except ValueError:
            continue
        if doc.get("msg") != DRY_RUN_MSG:
            continue
        cls = ""
        details = doc.get("algorithmFailureDetails")
        if isinstance(details, str) and details.startswith("{"):
            try:
                cls = (json.loads(details) or {}).get("class") or ""
            except ValueError:
                cls = ""
        out[(doc.get("algorithm") or "", doc.get("requestId") or "")] = {
            "stage": doc.get("stage"), "class": cls or ("running" if doc.get("stage") == "RUNNING" else "plain"),
            "time": doc.get("time", "")}
    return out


async def report(shadow: Dict[Tuple[str, str], Dict[str, Any]], store, limit: int = 50) -> Dict[str, Any]:
    counts = {"agree": 0, "differ": 0, "unfinished": 0, "missing": 0}
    by_class: Dict[str, Dict[str, int]] = {}
    differ: List[Dict[str, Any]] = []
    keys = list(shadow)
    rows: List[Any] = []
    for i in range(0, len(keys), 256):
        rows += await asyncio.gather(*(store.read_status(a, r) for a, r in keys[i:i + 256]))
    for (alg, rid), row in zip(keys, rows):
        rec = shadow[(alg, rid)]
        if row is None:
            what = "missing"
        elif row.lifecycle_stage == rec["stage"]:
            what = "agree"
        elif row.lifecycle_stage not in _cp.FINISHED_STAGES:
            what = "unfinished"
        else:
            what = "differ"
            if len(differ) < limit:
                differ.append({"algorithm": alg, "request_id": rid, "shadow_stage": rec["stage"],
                               "shadow_class": rec["class"], "store_stage": row.lifecycle_stage})
        counts[what] += 1
        c = by_class.setdefault(rec["class"], {"agree": 0, "differ": 0, "unfinished": 0, "missing": 0})
        c[what] += 1
    decided = counts["agree"] + counts["differ"]
    return {"runs": len(keys), **counts, "agreement": round(counts["agree"] / decided, 4) if decided else None,
            "by_class": by_class, "differences": differ}


def main(argv: List[str]) -> int:
    from .app import build_store
    from .config import load_config

    if not argv:
        print("usage: python -m nexus_supervisor_amd shadow-report LOG [LOG ...]   (the shadow supervisor's JSON log)",
              file=sys.stderr)
        return 2
    shadow: Dict[Tuple[str, str], Dict[str, Any]] = {}
    for path in argv:
        with (sys.stdin if path == "-" else open(path)) as f:
            shadow.update(parse_shadow_log(f))
    cfg = load_config()
    cfg.stages.apply()

    async def go():
        store = build_store(cfg)
        await store.connect()
        try:
            return await report(shadow, store)
        finally:
            await store.close()

    print(json.dumps(asyncio.run(go()), indent=2))
    return 0
