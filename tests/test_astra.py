"""Astra path (``cql-store-type: astra``, ``/root/reference/app/app_dependencies.go:18-25``):
Secure Connect Bundle → mutual TLS → metadata service → SNI proxy → CQL.

A local stand-in for Astra: an HTTPS metadata service and a TLS SNI proxy (client
certificates required, both signed by a throwaway CA made with ``openssl``) in front
of the native CQL server."""
import asyncio
import base64
import io
import json
import os
import shutil
import ssl
import subprocess
import zipfile

import pytest

from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.store.cql import CqlCheckpointStore, load_secure_bundle
from nexus_supervisor_amd.testing.cqlsrv import CqlServer
from nexus_supervisor_amd.testing.seed import ALGORITHM, seed_cql_statements, seed_rows

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI needed to mint certificates")


def _sh(*args, cwd):
    subprocess.run(list(args), cwd=cwd, check=True, capture_output=True)


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = tmp_path_factory.mktemp("pki")
    _sh("openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-out", "ca.crt", "-days", "2",
        "-subj", "/CN=test-astra-ca", cwd=d)
    for name, cn in (("server", "127.0.0.1"), ("client", "nexus-supervisor")):
        _sh("openssl", "req", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{name}.key", "-out", f"{name}.csr",
            "-subj", f"/CN={cn}", cwd=d)
        (d / f"{name}.ext").write_text("subjectAltName=IP:127.0.0.1\n")
        _sh("openssl", "x509", "-req", "-in", f"{name}.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial",
            "-out", f"{name}.crt", "-days", "2", "-extfile", f"{name}.ext", cwd=d)
    return d


def _server_ctx(pki, seen_sni):
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(str(pki / "server.crt"), str(pki / "server.key"))
    ctx.load_verify_locations(str(pki / "ca.crt"))
    ctx.verify_mode = ssl.CERT_REQUIRED

    def sni(sslobj, name, _ctx):
        seen_sni.append(name)

    ctx.sni_callback = sni
    return ctx


async def _sni_proxy(ctx, backend_port):
    async def handle(r, w):
        try:
            br, bw = await asyncio.open_connection("127.0.0.1", backend_port)
        except OSError:
            w.close()
            return

        async def pump(src, dst):
            try:
                while True:
                    data = await src.read(65536)
                    if not data:
                        break
                    dst.write(data)
                    await dst.drain()
            except (ConnectionError, asyncio.CancelledError):
                pass
            finally:
                dst.close()

        await asyncio.gather(pump(r, bw), pump(br, w))

    return await asyncio.start_server(handle, "127.0.0.1", 0, ssl=ctx)


async def _metadata_service(ctx, proxy_port, host_ids):
    async def handle(r, w):
        await r.readuntil(b"\r\n\r\n")
        body = json.dumps({"version": 1, "region": "local", "contact_info": {
            "type": "sni_proxy", "local_dc": "dc1", "contact_points": host_ids,
            "sni_proxy_address": f"127.0.0.1:{proxy_port}"}}).encode()
        w.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %d\r\nConnection: close\r\n\r\n"
                % len(body) + body)
        await w.drain()
        w.close()

    return await asyncio.start_server(handle, "127.0.0.1", 0, ssl=ctx)


def _bundle(pki, meta_port, proxy_port) -> str:
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        z.writestr("config.json", json.dumps({"host": "127.0.0.1", "port": meta_port, "cql_port": proxy_port,
                                              "keyspace": "nexus", "localDC": "dc1"}))
        z.write(pki / "ca.crt", "ca.crt")
        z.write(pki / "client.crt", "cert")
        z.write(pki / "client.key", "key")
    return base64.b64encode(buf.getvalue()).decode()


def test_secure_connect_bundle_end_to_end(pki, arun):
    host_id = "4f0f2d6e-6a55-4c4f-9f8e-4b3c1d2e0a11"
    with CqlServer(exec_statements=seed_cql_statements(), user="token", password="AstraCS:secret") as srv:
        async def go():
            seen = []
            ctx = _server_ctx(pki, seen)
            proxy = await _sni_proxy(ctx, srv.port)
            pport = proxy.sockets[0].getsockname()[1]
            meta = await _metadata_service(ctx, pport, [host_id])
            mport = meta.sockets[0].getsockname()[1]
            b64 = _bundle(pki, mport, pport)
            parsed = load_secure_bundle(b64)
            assert parsed.host == "127.0.0.1" and parsed.cql_port == pport and parsed.local_dc == "dc1"
            cfg = load_config(path=None, env={"NEXUS__ASTRA_CQL_STORE__SECURE_CONNECTION_BUNDLE_BASE64": b64,
                                              "NEXUS__ASTRA_CQL_STORE__GATEWAY_USER": "token",
                                              "NEXUS__ASTRA_CQL_STORE__GATEWAY_PASSWORD": "AstraCS:secret"},
                              overrides={"cql-store-type": "astra"})
            store = CqlCheckpointStore.from_config(cfg)
            await store.connect()
            row = await store.read_checkpoint(ALGORITHM, seed_rows()[0].id)
            assert row == seed_rows()[0]
            assert host_id in seen  # node connections are routed by SNI = host id
            await store.close()
            proxy.close()
            meta.close()

        arun(go(), timeout=60)


def test_bundle_without_ca_is_rejected():
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        z.writestr("config.json", "{}")
    with pytest.raises(Exception):
        load_secure_bundle(base64.b64encode(buf.getvalue()).decode())
