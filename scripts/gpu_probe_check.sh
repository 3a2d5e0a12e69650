#!/bin/bash
# First hardware check of the HIP probe kernels (selftest, probe at several sizes, rocprof stats).
set -u
O=gpurun_out/probe1
mkdir -p $O
B=build/native
timeout -k 10 60 $B/probe_selftest > $O/selftest.txt 2>&1; echo "selftest rc=$?" >> $O/selftest.txt
timeout -k 10 60 $B/mi355x-probe --list > $O/list.txt 2>&1 || exit 1
timeout -k 10 120 $B/mi355x-probe --hbm-bytes 268435456 --gemm-n 1024 > $O/probe_small.json 2>&1 || exit 1
timeout -k 10 120 $B/mi355x-probe > $O/probe_1g.json 2>&1 || exit 1
timeout -k 10 180 $B/mi355x-probe --hbm-bytes 17179869184 --gemm-n 8192 > $O/probe_16g.json 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o probe -- $GRAFT_REPO_ROOT/$B/mi355x-probe > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
echo "rocprof rc=$?" >> $GRAFT_REPO_ROOT/$O/prof.log
