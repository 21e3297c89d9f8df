#!/bin/bash
# fp32 page staging: one LDS round (exp build) vs two (default), isolated C5 A and B.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/lib_ab.sh exp/lib_r32_1.so c5 || exit $?
