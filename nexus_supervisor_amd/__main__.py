"""Command line: ``python -m nexus_supervisor_amd <command>``.

``supervisor``  the cluster supervisor (default; reference ``main.go``)
``agent``       the per-node GPU attribution agent (needs ``NODE_NAME``)
``worker``      one shard-worker process (spawned by the supervisor when
                ``runtime.worker-processes`` > 1; not started by hand)
``config``      print the effective configuration (secrets masked)
``explain``     what the supervisor would decide for ``kubectl get … -o json`` output, and why
``shadow-report`` how a dry-run (shadow) supervisor's decisions agree with the checkpoint store
``build``       build the native components in-tree
``cqlsrv``      run the native in-memory CQL server (tests / local runs)
``version``     print the version
"""
from __future__ import annotations

import json
import os
import subprocess
import sys


def main(argv=None) -> int:
    from .utils.covtrace import install_from_env

    install_from_env()  # child-process coverage for tools/coverage_gate.py (no-op unless enabled)
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = argv.pop(0) if argv and not argv[0].startswith("-") else "supervisor"
    if cmd == "supervisor":
        from .app import main as run

        return run(argv)
    if cmd == "worker":
        from .parallel.workers import worker_main

        return worker_main()
    if cmd == "agent":
        import asyncio

        from .config import load_config
        from .gpu.agent import run_agent
        from .obs.logging import configure_logging

        cfg = load_config()
        configure_logging(cfg.log_level, static={"service": "nexus-gpu-agent"})
        node = os.environ.get("NODE_NAME", "")
        if not node:
            print("NODE_NAME is required (downward API spec.nodeName)", file=sys.stderr)
            return 1
        asyncio.run(run_agent(cfg, node))
        return 0
    if cmd == "config":
        from .config import load_config, redacted

        print(json.dumps(redacted(load_config()), indent=2, default=str))
        return 0
    if cmd == "explain":
        from .explain import main as explain

        return explain(argv)
    if cmd == "shadow-report":
        from .shadow import main as shadow_report

        return shadow_report(argv)
    if cmd == "build":
        from ._build import main as build

        return build(argv)
    if cmd == "cqlsrv":
        from ._build import binary

        # child process (never exec): keeps signal handling simple for callers
        return subprocess.call([binary("nexus-cqlsrv")] + argv)
    if cmd == "version":
        from .buildmeta import main as version

        return version(argv)
    print(__doc__, file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())
