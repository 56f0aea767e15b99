#!/bin/bash
# Build libquorumbatch.so of a git revision (default HEAD) into
# tools/lab/ab/<name>.so for the A/B scripts (ab_rows.sh, ab_tracker.sh,
# prof_libs.sh), from a temporary worktree so the working tree is untouched.
#   tools/lab/build_ref_lib.sh [rev] [name]      Development tool.
set -e
cd "$(dirname "$0")/../.."
rev=${1:-HEAD}; name=${2:-head}
wt=$(mktemp -d /tmp/qb_ref_XXXXXX)
git worktree add -q --detach "$wt" "$rev"
trap 'git worktree remove --force "$wt"' EXIT
make -C "$wt/etcd_amd/csrc" -s -j8
mkdir -p tools/lab/ab
cp "$wt/etcd_amd/libquorumbatch.so" "tools/lab/ab/$name.so"
echo "tools/lab/ab/$name.so <- $(git rev-parse --short "$rev")"
