#!/bin/bash
# Measured int32 VALU issue rate (the Keccak roofline's peak); compiled on the box.
set -o pipefail
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/valu_peak scripts/valu_peak.hip && \
timeout -k 10 60 gpurun_out/valu_peak | tee gpurun_out/valu_peak.txt
