"""Container log tails: the OOM text a default pod never puts in its termination message.

Kubernetes fills ``containerStatuses[].state.terminated.message`` only from the
container's ``terminationMessagePath`` (``/dev/termination-log``) under the default
``terminationMessagePolicy: File``.  PyTorch never writes that file: a torch HBM-OOM
prints ``torch.OutOfMemoryError: HIP out of memory. Tried to allocate …`` to stderr and
exits 1, so on a default pod the only place the signature lives is the container log.
(The reference learns of OOMs from the Job controller's ``PodFailurePolicy`` event
message, ``/root/reference/services/supervisor.go:194-204,311-312``, which never says
*which* memory ran out.)

Two readers, one scanner:

* **node agent** — reads ``/var/log/pods/<ns>_<pod>_<uid>/<container>/<restart>.log``
  (the kubelet's CRI log layout; docker ``json-file`` lines are understood too) from a
  read-only hostPath mount: :func:`read_container_tail`;
* **supervisor** — ``GET /api/v1/namespaces/<ns>/pods/<pod>/log?container=…&tailLines=…
  &limitBytes=…[&previous=true]`` (RBAC ``pods/log get``): :func:`fetch_api_tail`.

:func:`scan` keeps only what matters from a tail: the lines that carry an HBM or host
allocation-failure signature (:mod:`.oom`), at most a few, each clipped — the tail itself
never travels into the checkpoint row.
"""
from __future__ import annotations

import glob
import json
import os
import re
from typing import Any, Dict, List, Optional, Tuple

from ..models import kube

from . import oom

LOG_ROOT = "/var/log/pods"
TAIL_BYTES = 64 * 1024
TAIL_LINES = 200
MAX_HITS = 3
LINE_CLIP = 600

# CRI log line: "<RFC3339Nano> <stdout|stderr> <P|F> <content>" (P = partial line)
_CRI = re.compile(rb"^(\S+) (stdout|stderr) ([PF]) ?(.*)$")


def parse_log_lines(data: bytes) -> List[str]:
    """Decode a chunk of a container log (CRI or docker json-file; anything else is taken
    as plain text) into whole lines, partial CRI records (``P``) re-joined."""
    out: List[str] = []
    partial: List[bytes] = []
    for raw in data.split(b"\n"):
        if not raw:
            continue
        m = _CRI.match(raw)
        if m is not None:
            partial.append(m.group(4))
            if m.group(3) == b"F":
                out.append(b"".join(partial).decode("utf-8", "replace"))
                partial = []
            continue
        if raw[:1] == b"{":
            try:
                doc = json.loads(raw)
            except ValueError:
                doc = None
            if isinstance(doc, dict) and isinstance(doc.get("log"), str):
                out.append(doc["log"].rstrip("\n"))
                continue
        out.append(raw.decode("utf-8", "replace"))
    if partial:
        out.append(b"".join(partial).decode("utf-8", "replace"))
    return out


def read_tail(path: str, max_bytes: int = TAIL_BYTES, max_lines: int = TAIL_LINES) -> List[str]:
    """Last ``max_lines`` lines within the last ``max_bytes`` of a log file (the first,
    possibly cut, line of the window is dropped)."""
    with open(path, "rb") as f:
        f.seek(0, os.SEEK_END)
        size = f.tell()
        start = max(0, size - max_bytes)
        f.seek(start)
        data = f.read(size - start)
    if start > 0:
        nl = data.find(b"\n")
        data = data[nl + 1:] if nl >= 0 else b""
    return parse_log_lines(data)[-max_lines:]


def _safe_part(s: str) -> bool:
    """A path component from the API (namespace, pod, uid, container name): Kubernetes
    validates them as DNS labels / UUIDs, but the agent runs privileged, so a name that could
    leave ``/var/log/pods`` is refused rather than trusted."""
    return bool(s) and "/" not in s and "\\" not in s and "\x00" not in s and s not in (".", "..")


def container_log_dir(root: str, namespace: str, pod: str, uid: str, container: str) -> Optional[str]:
    if not all(_safe_part(x) for x in (namespace, pod, uid, container)):
        return None
    return os.path.join(root, f"{namespace}_{pod}_{uid}", container)


def _unreadable_dir(d: str) -> bool:
    """``d`` (or a parent under the log root) exists but this process may not list it."""
    while d and d != os.path.dirname(d):
        try:
            os.stat(d)
        except PermissionError:
            return True
        except OSError:
            d = os.path.dirname(d)
            continue
        return os.path.isdir(d) and not os.access(d, os.R_OK | os.X_OK)
    return False


def container_log_file(root: str, namespace: str, pod: str, uid: str, container: str,
                       restart: Optional[int] = None) -> Optional[str]:
    """The kubelet's file for one container instance: ``<restart>.log``; without an exact
    match, the newest ``N.log`` of the container (rotated files are not read: the failure
    is at the end of the live file)."""
    d = container_log_dir(root, namespace, pod, uid, container)
    if d is None:
        return None
    if restart is not None:
        p = os.path.join(d, f"{int(restart)}.log")
        if os.path.isfile(p):
            return p
    best, best_n = None, -1
    for p in glob.glob(os.path.join(glob.escape(d), "*.log")):
        stem = os.path.basename(p)[:-4]
        if stem.isdigit() and int(stem) > best_n:
            best, best_n = p, int(stem)
    return best


def scan(lines: List[str]) -> Dict[str, Any]:
    """The allocation-failure lines of a tail, newest last: ``{"match": "hbm"|"host"|None,
    "lines": [...]}``.  An HBM signature anywhere in the tail wins over a host one (a torch
    OOM traceback is followed by nothing but the interpreter's exit)."""
    hits: List[Tuple[str, str]] = []
    for line in lines:
        if oom.hbm_signature(line):
            hits.append(("hbm", line))
        elif oom.host_signature(line):
            hits.append(("host", line))
    kinds = {k for k, _ in hits}
    match = "hbm" if "hbm" in kinds else "host" if "host" in kinds else None
    # prefer the lines of the winning kind; the torch line naming the GPU and its capacity
    # is the one that says most, keep it even when a later line also matches
    chosen = [ln for k, ln in hits if k == match]
    torch_lines = [ln for ln in chosen if "total capacity" in ln.lower()]
    keep = (torch_lines[-1:] + [ln for ln in chosen if ln not in torch_lines[-1:]])[-MAX_HITS:] if chosen else []
    return {"match": match, "lines": [ln[-LINE_CLIP:] for ln in keep]}


def failed_containers(pod: Dict[str, Any]) -> List[Dict[str, Any]]:
    """Failed container instances of a pod worth a log read: non-zero exit, not a cgroup
    OOMKill (already a kernel fact), and an empty termination message (otherwise the
    message *is* the log's last words).  ``restart`` is the instance's log file number
    (``state`` → restartCount, ``lastState`` → restartCount − 1); ``previous`` is what
    the pods/log API needs to reach that instance."""
    out = []
    for cs in kube.container_statuses(pod):
        rc = int(cs.get("restartCount") or 0)
        for which in ("state", "lastState"):
            t = (cs.get(which) or {}).get("terminated")
            if not t:
                continue
            if (t.get("exitCode") or 0) == 0 or t.get("reason") == "OOMKilled" or (t.get("message") or "").strip():
                continue
            prev = which == "lastState"
            out.append({"container": cs.get("name", ""), "restart": max(0, rc - 1) if prev else rc, "previous": prev,
                        "exitCode": t.get("exitCode")})
            break  # the current instance's failure, or else the last one's: one read per container
    return out


def node_log_evidence(root: str, pod: Dict[str, Any], max_bytes: int = TAIL_BYTES) -> List[Dict[str, Any]]:
    """Node-agent reader: one record per failed container (``match`` None when the tail
    was read and carries no signature — the supervisor then need not fetch it again)."""
    ns, name, uid = kube.namespace_of(pod), kube.name_of(pod), kube.uid_of(pod)
    out = []
    for fc in failed_containers(pod):
        path = container_log_file(root, ns, name, uid, fc["container"], fc["restart"])
        rec: Dict[str, Any] = {"container": fc["container"], "restart": fc["restart"], "source": "node-log"}
        if path is None:
            d = container_log_dir(root, ns, name, uid, fc["container"])
            if d is not None and _unreadable_dir(d):
                rec["error"] = "PermissionError: log directory not readable"
                rec["denied"] = True
            else:
                rec["error"] = "no log file"
        else:
            try:
                rec.update(scan(read_tail(path, max_bytes)))
            except OSError as exc:
                rec["error"] = f"{type(exc).__name__}: {exc.strerror or exc}"
                if isinstance(exc, PermissionError):
                    rec["denied"] = True  # root-owned 0640 kubelet logs and a non-root reader
        out.append(rec)
    return out


async def fetch_api_tail(client, namespace: str, pod: str, container: str, previous: bool = False,
                         tail_lines: int = TAIL_LINES, limit_bytes: int = TAIL_BYTES,
                         timeout: float = 2.0) -> Dict[str, Any]:
    """Supervisor reader over ``pods/<pod>/log``; same record shape as the node reader."""
    rec: Dict[str, Any] = {"container": container, "source": "pods/log"}
    try:
        status, body = await client.pod_log(namespace, pod, container, previous=previous, tail_lines=tail_lines,
                                            limit_bytes=limit_bytes, timeout=timeout)
    except Exception as exc:  # noqa: BLE001 - a log is evidence, never a reason to fail
        rec["error"] = f"{type(exc).__name__}: {exc}"[:200]
        return rec
    if status >= 400:
        rec["error"] = f"HTTP {status}"
        return rec
    rec.update(scan(parse_log_lines(body)[-tail_lines:]))
    return rec


def log_texts(records) -> List[Tuple[str, str]]:
    """``(source, line)`` pairs for :func:`.oom.analyze` from log records."""
    out = []
    for r in records or ():
        if not isinstance(r, dict):
            continue
        src = f"{r.get('source', 'log')} tail of container {r.get('container', '')}"
        for ln in r.get("lines") or ():
            out.append((src, ln))
    return out
