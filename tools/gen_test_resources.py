#!/usr/bin/env python3
"""Write ``deploy/test-resources/checkpoints.cql`` (schema + the 8 seed rows) from
``testing/seed.py`` — the file the docker-compose Scylla setup applies (reference:
``test-resources/checkpoints.cql`` + ``prepare-scylla.sh``)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nexus_supervisor_amd.testing.seed import seed_cql_statements  # noqa: E402

OUT = os.path.join(ROOT, "deploy", "test-resources", "checkpoints.cql")


def render() -> str:
    stmts = [s for s in seed_cql_statements() if not s.lstrip().upper().startswith("CREATE KEYSPACE")]
    return "\n\n".join(s.rstrip().rstrip(";") + ";" for s in stmts) + "\n"


if __name__ == "__main__":
    with open(OUT, "w") as f:
        f.write(render())
    print(OUT)
