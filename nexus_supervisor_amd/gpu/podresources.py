"""Kubelet pod-resources client: which GPU devices each pod container was allocated.

The AMD device plugin allocates ``amd.com/gpu`` devices by PCI address; the
kubelet exposes the allocation on ``/var/lib/kubelet/pod-resources/kubelet.sock``
(gRPC service ``v1.PodResourcesLister``).  The node agent joins it with the
amd-smi BDF of each GPU to attribute a failing pod to physical GPUs without
relying on the pod's env.  The protobuf messages are tiny, so they are encoded
and decoded by hand (no generated stubs are available offline):

    ListPodResourcesResponse { repeated PodResources pod_resources = 1; }
    PodResources { string name = 1; string namespace = 2; repeated ContainerResources containers = 3; }
    ContainerResources { string name = 1; repeated ContainerDevices devices = 2; }
    ContainerDevices { string resource_name = 1; repeated string device_ids = 2; }
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Tuple

SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
LIST_METHOD = "/v1.PodResourcesLister/List"


def _varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7


def _fields(b: bytes) -> Iterator[Tuple[int, object]]:
    i = 0
    while i < len(b):
        k, i = _varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _varint(b, i)
            yield f, v
        elif wt == 2:
            n, i = _varint(b, i)
            yield f, b[i:i + n]
            i += n
        elif wt == 1:
            i += 8
        elif wt == 5:
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")


def decode_list_response(raw: bytes) -> List[Dict[str, object]]:
    pods = []
    for f, pr in _fields(raw):
        if f != 1:
            continue
        pod = {"name": "", "namespace": "", "containers": []}
        for pf, pv in _fields(pr):
            if pf == 1:
                pod["name"] = pv.decode()
            elif pf == 2:
                pod["namespace"] = pv.decode()
            elif pf == 3:
                c = {"name": "", "devices": []}
                for cf, cv in _fields(pv):
                    if cf == 1:
                        c["name"] = cv.decode()
                    elif cf == 2:
                        d = {"resource_name": "", "device_ids": []}
                        for df, dv in _fields(cv):
                            if df == 1:
                                d["resource_name"] = dv.decode()
                            elif df == 2:
                                d["device_ids"].append(dv.decode())
                        c["devices"].append(d)
                pod["containers"].append(c)
        pods.append(pod)
    return pods


def _enc_bytes(field: int, data: bytes) -> bytes:
    n = len(data)
    out = bytearray([(field << 3) | 2])
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            break
    return bytes(out) + data


def encode_list_response(pods: List[Dict[str, object]]) -> bytes:
    """Inverse of :func:`decode_list_response` (fake kubelet in tests)."""
    out = b""
    for p in pods:
        body = _enc_bytes(1, p["name"].encode()) + _enc_bytes(2, p["namespace"].encode())
        for c in p.get("containers", []):
            cb = _enc_bytes(1, c["name"].encode())
            for d in c.get("devices", []):
                db = _enc_bytes(1, d["resource_name"].encode())
                for did in d["device_ids"]:
                    db += _enc_bytes(2, did.encode())
                cb += _enc_bytes(2, db)
            body += _enc_bytes(3, cb)
        out += _enc_bytes(1, body)
    return out


ALLOCATABLE_METHOD = "/v1.PodResourcesLister/GetAllocatableResources"


def decode_allocatable_response(raw: bytes) -> List[Dict[str, object]]:
    """``AllocatableResourcesResponse { repeated ContainerDevices devices = 1; … }`` →
    ``[{"resource_name", "device_ids"}]`` (cpu_ids / memory are skipped)."""
    out = []
    for f, cv in _fields(raw):
        if f != 1:
            continue
        d = {"resource_name": "", "device_ids": []}
        for df, dv in _fields(cv):
            if df == 1:
                d["resource_name"] = dv.decode()
            elif df == 2:
                d["device_ids"].append(dv.decode())
        out.append(d)
    return out


def encode_allocatable_response(devices: List[Dict[str, object]]) -> bytes:
    """Inverse of :func:`decode_allocatable_response` (fake kubelet in tests)."""
    out = b""
    for d in devices:
        db = _enc_bytes(1, d["resource_name"].encode())
        for did in d["device_ids"]:
            db += _enc_bytes(2, did.encode())
        out += _enc_bytes(1, db)
    return out


def allocatable_ids(devices: List[Dict[str, object]], resource: str = "amd.com/gpu") -> List[str]:
    """Device ids of one resource the kubelet's device manager offers for allocation."""
    return [i for d in devices if d["resource_name"] == resource for i in d["device_ids"]]


def gpu_allocations(pods: List[Dict[str, object]], resource: str = "amd.com/gpu") -> Dict[Tuple[str, str], List[str]]:
    """``(namespace, pod) -> [device ids]`` for one resource."""
    out: Dict[Tuple[str, str], List[str]] = {}
    for p in pods:
        ids = [i for c in p["containers"] for d in c["devices"] if d["resource_name"] == resource for i in d["device_ids"]]
        if ids:
            out[(p["namespace"], p["name"])] = ids
    return out


class PodResourcesClient:
    def __init__(self, socket_path: str = SOCKET, timeout: float = 5.0):
        self.target = f"unix://{socket_path}"
        self.timeout = timeout
        self._channel = None

    def list(self) -> List[Dict[str, object]]:
        import grpc

        if self._channel is None:
            self._channel = grpc.insecure_channel(self.target)
        call = self._channel.unary_unary(LIST_METHOD, request_serializer=lambda _: b"",
                                         response_deserializer=lambda b: b)
        return decode_list_response(call(None, timeout=self.timeout))

    def allocatable(self) -> List[Dict[str, object]]:
        """``GetAllocatableResources`` (kubelet ≥ 1.23): the devices the device manager
        offers — a GPU the AMD device plugin reported unhealthy is missing from it."""
        import grpc

        if self._channel is None:
            self._channel = grpc.insecure_channel(self.target)
        call = self._channel.unary_unary(ALLOCATABLE_METHOD, request_serializer=lambda _: b"",
                                         response_deserializer=lambda b: b)
        return decode_allocatable_response(call(None, timeout=self.timeout))

    def check(self) -> str:
        """``ok``, ``missing`` or ``denied``: can this process connect to the kubelet's
        socket at all (root-only on a default kubelet; gRPC would only say UNAVAILABLE)."""
        import socket as _socket

        path = self.target[len("unix://"):]
        s = _socket.socket(_socket.AF_UNIX, _socket.SOCK_STREAM)
        try:
            s.settimeout(self.timeout)
            s.connect(path)
            return "ok"
        except PermissionError:
            return "denied"
        except FileNotFoundError:
            return "missing"
        except OSError as exc:
            return f"error: {exc.strerror or exc}"
        finally:
            s.close()

    def close(self) -> None:
        if self._channel is not None:
            self._channel.close()
            self._channel = None


def normalize_bdf(dev_id: str) -> str:
    """Device-plugin ids are PCI addresses (``0000:0a:00.0``); tolerate a missing domain."""
    d = dev_id.strip().lower()
    if d.count(":") == 1:
        d = "0000:" + d
    return d
