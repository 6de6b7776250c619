# r02: executor overlap timelines at 256 MiB per rank (8-rank loopback world, reference loop sizes)
set -o pipefail
export HCCL_BUFFSIZE=200 TRACE_MIB=256 TRACE_CALLS=3
TRACE_ALGO=MESH_TWOSHOT bash tools/trace_loopback.sh r02_twoshot256 && \
TRACE_ALGO=MESH_CHUNK bash tools/trace_loopback.sh r02_meshchunk256 && \
TRACE_ALGO=RING bash tools/trace_loopback.sh r02_ring256
