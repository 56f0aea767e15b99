#!/bin/bash
# Lab: the leader step's message stores as five 8-byte stores (no streaming hint)
# (tools/lab/ab/wordmsg.so) against the tree, on the leader and ReadIndex rows
# (DESIGN §3.7c).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/lab/ab_rows.sh 3 readindex tree wordmsg > $O/ab_readindex_wordmsg.log 2>&1 || exit 1
bash tools/lab/ab_rows.sh 2 leader tree wordmsg > $O/ab_leader_wordmsg.log 2>&1 || exit 1
cat $O/*.log
