set -o pipefail
O=gpurun_out/r4_36
mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result bench/probes/mfma_shape_probe.hip -o /tmp/mfma_probe && \
timeout -k 10 120 /tmp/mfma_probe > $O/mfma_shape.log 2>&1
