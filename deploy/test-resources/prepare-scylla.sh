#!/usr/bin/env bash
# Create the nexus keyspace and apply the checkpoint schema + seed rows to a local Scylla
# (docker-compose `prepare_scylla` service).
set -euo pipefail
HOST="${CQL_HOST:-localhost}"
cqlsh "$HOST" -e "CREATE KEYSPACE IF NOT EXISTS nexus WITH replication = { 'class': 'SimpleStrategy', 'replication_factor': 1 };"
echo 'Applying checkpoints table'
cqlsh "$HOST" -f /opt/storage/checkpoints.cql
echo 'Checking table'
cqlsh "$HOST" -e 'SELECT algorithm, id, lifecycle_stage FROM nexus.checkpoints'
