#!/bin/bash
# GPU: interleaved A/B timing with the opt-in dS path enabled (FA2_DS_WORKSPACE_MAX_GB=auto).
# usage: ab_env.sh TAG WHAT CAUSAL libs...
set -o pipefail
TAG=$1; WHAT=$2; CAUSAL=$3; shift 3
mkdir -p gpurun_out/$TAG
FA2_DS_WORKSPACE_MAX_GB=auto WHAT=$WHAT CAUSAL=$CAUSAL timeout -k 10 300 python scripts/ab.py "$@" > gpurun_out/$TAG/ab.log 2>&1; rc=$?
cat gpurun_out/$TAG/ab.log; exit $rc
