#!/bin/bash
# Snapshot a git ref as _ab/base/ for on-box A/B runs (tools/gpu.sh hotpath / basebench).
#
#   bash tools/ab_snapshot.sh [REF]          (default HEAD)
#
# The package, native sources, bench.py and tools of REF; the native builds are copied from
# the working tree (valid when REF's native sources equal the tree's — the script checks
# and refuses otherwise) and stripped of debug info so the upload stays small.
set -euo pipefail
cd "$(dirname "$0")/.."
ref=${1:-HEAD}
if ! git diff --quiet "$ref" -- csrc; then
  echo "csrc differs between $ref and the working tree: build $ref's natives first" >&2
  exit 1
fi
rm -rf _ab/base
mkdir -p _ab/base
git archive "$ref" nexus_supervisor_amd csrc bench.py tools | tar -x -C _ab/base
cp tools/hotpath_bench.py _ab/base/tools/  # the harness itself comes from the tree
(cd nexus_supervisor_amd && find . \( -name "*.so" -o -path "./bin/*" \) -type f \
   ! -name "*-address" ! -name "*-undefined" ! -name "*-thread") | while read -r f; do
  mkdir -p "_ab/base/nexus_supervisor_amd/$(dirname "$f")"
  cp -p "nexus_supervisor_amd/$f" "_ab/base/nexus_supervisor_amd/$f"
  strip --strip-debug "_ab/base/nexus_supervisor_amd/$f" 2>/dev/null || true
done
# the copies must not look older than the sources (the build's up-to-date check)
find _ab/base/nexus_supervisor_amd \( -name "*.so" -o -path "*/bin/*" \) -type f -exec touch {} +
du -sh _ab
