"""Self-signed certificate bootstrap for the shard-label webhook
(``sharding.webhook-cert-bootstrap``).

The API server calls the webhook over HTTPS and trusts it through the
``MutatingWebhookConfiguration``'s ``caBundle``.  With cert-manager, the chart mounts the
issued Secret and the operator sets ``caBundle`` (``deploy/helm``); without it this module
does both, so the webhook never silently stops being called because of a certificate
nobody renewed (``failurePolicy: Ignore`` turns that into unlabelled Jobs — repaired by
the audit, :class:`..admission.ShardLabelKeeper`, but only an interval later):

1. every replica reads the Secret ``webhook-secret`` (``tls.crt``, ``tls.key``, ``ca.crt``);
2. when it is missing, unreadable, for other DNS names, or within ``renew-before`` of its
   expiry, the replica mints a new CA + serving certificate (:mod:`._certgen`, libcrypto)
   and writes the Secret with a compare-and-swap (create → 409, or update at the
   resourceVersion it read → 409): one replica wins, the others re-read and use its pair;
3. the pair is written to the webhook's certificate directory (the server reloads it,
   :meth:`..admission.WebhookServer.check_cert`);
4. every webhook of ``webhook-config-name`` gets ``caBundle`` = the current CA followed by
   the previous one (a rotation overlaps: an API server still holding the old bundle, a
   replica still serving the old certificate) — GET + PUT at its resourceVersion.

RBAC: Secrets get/create/update (namespaced, the one name) and
mutatingwebhookconfigurations get/update (cluster-scoped, the one name) — the chart's
``sharding.webhook.certBootstrap``.  No counterpart in the reference (it has no webhook).
"""
from __future__ import annotations

import asyncio
import base64
import os
import ssl
import tempfile
import time
from typing import Any, Dict, List, Optional, Tuple

from .kube.errors import ApiError

DAY = 86400.0


def _b64(s: str) -> str:
    return base64.b64encode(s.encode()).decode()


def _unb64(s: Optional[str]) -> str:
    return base64.b64decode(s or "").decode() if s else ""


def decode_cert(pem: str) -> Optional[Dict[str, Any]]:
    """``ssl``'s decoded view of the first certificate of a PEM string (subject, SAN,
    notAfter), None when it does not parse."""
    if "BEGIN CERTIFICATE" not in pem:
        return None
    fd, path = tempfile.mkstemp(suffix=".pem")
    try:
        with os.fdopen(fd, "w") as f:
            f.write(pem)
        return ssl._ssl._test_decode_cert(path)  # noqa: SLF001 - the stdlib's own PEM → dict
    except (OSError, ssl.SSLError, ValueError):
        return None
    finally:
        os.unlink(path)


def _first_pem(bundle: str) -> str:
    end = "-----END CERTIFICATE-----"
    i = bundle.find(end)
    return bundle[:i + len(end)] + "\n" if i >= 0 else ""


def webhook_dns_names(service: str, namespace: str) -> List[str]:
    """The names the API server dials a webhook Service by."""
    return [f"{service}.{namespace}.svc", f"{service}.{namespace}.svc.cluster.local", f"{service}.{namespace}"]


class WebhookCertBootstrap:
    def __init__(self, kube, namespace: str, secret: str, config_name: str, service: str, cert_dir: str, *,
                 days: int = 365, renew_before: float = 30 * DAY, metrics=None, log=None,
                 clock=time.time):
        self.kube = kube
        self.namespace = namespace
        self.secret = secret
        self.config_name = config_name
        self.dns = webhook_dns_names(service, namespace)
        self.cert_dir = cert_dir
        self.days = days
        self.renew_before = renew_before
        self.metrics = metrics
        self.log = log
        self.clock = clock
        self.minted = 0
        self.ca_patches = 0
        self._task: Optional[asyncio.Task] = None

    @classmethod
    def from_config(cls, cfg, kube, metrics=None, log=None) -> "WebhookCertBootstrap":
        s = cfg.sharding
        return cls(kube, cfg.resource_namespace, s.webhook_secret, s.webhook_config_name, s.webhook_service,
                   s.webhook_cert_dir, metrics=metrics, log=log)

    # ------------------------------------------------------------------ the Secret
    def _usable(self, data: Dict[str, str]) -> bool:
        crt, key = _unb64(data.get("tls.crt")), _unb64(data.get("tls.key"))
        if not crt or "PRIVATE KEY" not in key:
            return False
        info = decode_cert(crt)
        if not info:
            return False
        sans = {v for k, v in info.get("subjectAltName", ()) if k == "DNS"}
        if not set(self.dns[:2]) <= sans:
            return False
        try:
            not_after = ssl.cert_time_to_seconds(info["notAfter"])
        except (KeyError, ValueError):
            return False
        return not_after - self.clock() > self.renew_before

    def _mint(self, previous_ca: str) -> Dict[str, str]:
        from . import _certgen

        ca, crt, key = _certgen.mint("nexus-supervisor-webhook-ca", self.dns, self.days)
        self.minted += 1
        if self.metrics is not None:
            self.metrics.inc("webhook_certs_minted")
        # the bundle the API server trusts: the new CA, then the one it replaces
        bundle = ca + (_first_pem(previous_ca) if previous_ca and _first_pem(previous_ca) != ca else "")
        return {"tls.crt": _b64(crt), "tls.key": _b64(key), "ca.crt": _b64(bundle)}

    async def _read_secret(self) -> Optional[Dict[str, Any]]:
        try:
            return await self.kube.get("Secret", self.namespace, self.secret)
        except ApiError as exc:
            if exc.status == 404:
                return None
            raise

    async def ensure_secret(self) -> Dict[str, str]:
        """The Secret's (decoded) ``tls.crt`` / ``tls.key`` / ``ca.crt``, minted and written
        first when missing or due for renewal; concurrent replicas converge on one pair."""
        for _ in range(5):
            cur = await self._read_secret()
            data = (cur or {}).get("data") or {}
            if cur is not None and self._usable(data):
                return {k: _unb64(v) for k, v in data.items()}
            fresh = self._mint(_unb64(data.get("ca.crt")))
            try:
                if cur is None:
                    await self.kube.create("Secret", self.namespace, {
                        "apiVersion": "v1", "kind": "Secret", "type": "kubernetes.io/tls",
                        "metadata": {"name": self.secret, "namespace": self.namespace,
                                     "labels": {"app.kubernetes.io/managed-by": "nexus-supervisor"}},
                        "data": fresh})
                else:
                    await self.kube.replace("Secret", self.namespace, self.secret, dict(cur, data=fresh))
            except ApiError as exc:
                if exc.status == 409:
                    continue  # another replica wrote first: use its pair
                raise
            if self.log is not None:
                self.log.info("webhook serving certificate minted", secret=self.secret, dns=self.dns[0])
            return {k: _unb64(v) for k, v in fresh.items()}
        raise RuntimeError(f"webhook certificate Secret {self.secret}: no stable version after 5 attempts")

    # ------------------------------------------------------------------ files + caBundle
    def write_files(self, pair: Dict[str, str]) -> bool:
        """``tls.crt`` / ``tls.key`` (and ``ca.crt``) into the certificate directory, each
        atomically; True when anything changed."""
        os.makedirs(self.cert_dir, exist_ok=True)
        changed = False
        for name in ("tls.key", "tls.crt", "ca.crt"):
            body = pair.get(name, "")
            path = os.path.join(self.cert_dir, name)
            try:
                with open(path) as f:
                    if f.read() == body:
                        continue
            except OSError:
                pass
            fd, tmp = tempfile.mkstemp(dir=self.cert_dir, prefix="." + name)
            with os.fdopen(fd, "w") as f:
                f.write(body)
            os.chmod(tmp, 0o600 if name == "tls.key" else 0o644)
            os.replace(tmp, path)
            changed = True
        return changed

    async def patch_ca_bundle(self, bundle: str) -> int:
        """Set every webhook's ``clientConfig.caBundle`` of the configuration to ``bundle``;
        returns how many changed (0 when already in step)."""
        want = _b64(bundle)
        for _ in range(5):
            try:
                cfg = await self.kube.get("MutatingWebhookConfiguration", None, self.config_name)
            except ApiError as exc:
                if exc.status == 404:
                    if self.log is not None:
                        self.log.warning("webhook configuration not found: caBundle not set", name=self.config_name)
                    return 0
                raise
            n = 0
            for wh in cfg.get("webhooks") or ():
                cc = wh.setdefault("clientConfig", {})
                if cc.get("caBundle") != want:
                    cc["caBundle"] = want
                    n += 1
            if not n:
                return 0
            try:
                await self.kube.replace("MutatingWebhookConfiguration", None, self.config_name, cfg)
            except ApiError as exc:
                if exc.status == 409:
                    continue
                raise
            self.ca_patches += 1
            if self.metrics is not None:
                self.metrics.inc("webhook_ca_bundle_updates")
            return n
        return 0

    async def sync(self) -> Tuple[bool, Dict[str, str]]:
        """One round: Secret → files → caBundle; returns (files changed, pair)."""
        pair = await self.ensure_secret()
        changed = self.write_files(pair)
        if self.config_name:
            await self.patch_ca_bundle(pair.get("ca.crt") or "")
        return changed, pair

    def start(self, interval: float = 3600.0, on_change=None) -> None:
        async def loop():
            while True:
                await asyncio.sleep(interval)
                try:
                    changed, _ = await self.sync()
                    if changed and on_change is not None:
                        on_change()
                except asyncio.CancelledError:
                    raise
                except Exception as exc:  # noqa: BLE001 - retried next interval; the expiry gauge alerts
                    if self.log is not None:
                        self.log.error(exc, "webhook certificate sync failed")

        self._task = asyncio.ensure_future(loop())

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            await asyncio.gather(self._task, return_exceptions=True)
            self._task = None
