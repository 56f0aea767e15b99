#!/bin/bash
# Lab: the leader step's message stores as five 8-byte streaming stores
# (tools/lab/ab/ntmsg.so) against the tree, on the leader and ReadIndex rows
# (DESIGN §3.7c).
set -o pipefail
O=${1:?outdir}; mkdir -p $O; export TMPDIR=/tmp
bash tools/lab/ab_rows.sh 3 readindex tree ntmsg > $O/ab_readindex_ntmsg.log 2>&1 || exit 1
bash tools/lab/ab_rows.sh 2 leader tree ntmsg > $O/ab_leader_ntmsg.log 2>&1 || exit 1
cat $O/*.log
