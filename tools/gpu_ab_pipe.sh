#!/bin/bash
# In-process knob A/B on the bench pipeline (tools/ab_pipeline.py), arguments passed through.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_pipeline.py "$@" > gpurun_out/ab_pipe.log 2>&1; rc=$?
cat gpurun_out/ab_pipe.log | grep -v amdgpu.ids; exit $rc
