#!/bin/bash
# Lab: the leader step without its message stores (tools/lab/ab/noemit.so,
# emit() counting only) against the tree — how much of the step the
# emission is.  Timing only; the lab build's messages are
# not written.
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/lab/ab_rows.sh 2 leader tree noemit > $O/ab_leader_noemit.log 2>&1 || exit 1
bash tools/lab/ab_rows.sh 2 readindex tree noemit > $O/ab_readindex_noemit.log 2>&1 || exit 1
cat $O/*.log
