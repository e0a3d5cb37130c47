#!/bin/bash
# build skb.hip variants (-D knobs) as small shared libraries and time the prep kernel alone
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/prep; mkdir -p $D
timeout -k 10 300 python -u tools/prep_probe.py tools/prep_so/base.so > $D/probe.log 2>&1; rc=$?
cat $D/probe.log | tail -5; exit $rc
