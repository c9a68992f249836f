#!/usr/bin/env bash
# BASELINE config 2 end to end on a kind cluster with a local Scylla (or nexus-cqlsrv):
#   1. kind cluster + namespace        3. supervisor (local process, kubeconfig of the cluster)
#   2. schema + BUFFERED rows           4. apply 100 failing Jobs, wait for every row's stage
# Needs: kind, kubectl, docker (compose), python with this package built.
set -euo pipefail
cd "$(dirname "$0")/../.."
PODS="${PODS:-100}"
CQL="${CQL:-127.0.0.1:9042}"
kind get clusters | grep -qx nexus || kind create cluster --config deploy/kind/cluster.yaml
kubectl create namespace nexus --dry-run=client -o yaml | kubectl apply -f -
docker compose -f deploy/docker-compose.yaml up -d scylla
docker compose -f deploy/docker-compose.yaml run --rm prepare_scylla
python -m nexus_supervisor_amd.bench.kindload seed --cql "$CQL" --pods "$PODS"
NEXUS_CONFIG_DIR=deploy APPLICATION_ENVIRONMENT=local NEXUS__KUBE_CONFIG_PATH="${KUBECONFIG:-$HOME/.kube/config}" \
  python -m nexus_supervisor_amd supervisor > /tmp/nexus-supervisor.log 2>&1 &
SUP=$!
trap 'kill $SUP' EXIT
until curl -sf http://127.0.0.1:8080/readyz > /dev/null; do sleep 0.5; done
python -m nexus_supervisor_amd.bench.kindload manifests --pods "$PODS" > /tmp/nexus-kindload.yaml
T_APPLY=$(python -c 'import time; print(time.time())')
kubectl apply -f /tmp/nexus-kindload.yaml > /dev/null
python -m nexus_supervisor_amd.bench.kindload wait --cql "$CQL" --pods "$PODS" --t-apply "$T_APPLY"
