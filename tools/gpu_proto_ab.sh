#!/bin/bash
# Protocol-tick A/B of libswarm builds on one box: tools/protocol_probe.py interleaved (hybrid 0.125,
# ROUNDS rounds), then a rocprofv3 kernel-trace summary of tools/protocol_pmc.py per library, then (PMC=1)
# the FETCH_SIZE / WRITE_SIZE passes of the first library.
#   LIBS="libswarm_old.so libswarm.so" ROUNDS=2 PMC=1 TAG=x bash tools/gpu_proto_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pab}
for i in $(seq 1 "${ROUNDS:-2}"); do
  for L in $LIBS; do
    timeout -k 10 200 python -u tools/protocol_probe.py --lib "$L" --modes hybrid:0.125 \
        | sed "s/^/$L /" || exit $?
  done
done
for L in $LIBS; do
  PROTO_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pk_${TAG}_${L%.so} -o run \
      -- python3 tools/protocol_pmc.py ${TAG}_${L%.so} > gpurun_out/pk_${TAG}_${L%.so}.log 2>&1 || exit $?
  f=$(find gpurun_out/pk_${TAG}_${L%.so} -name "*kernel_stats.csv" | head -1)
  echo "== $L"; grep -E "k_tick|k_pack|k_unpack|k_mail_from|k_kill" "$f" | cut -d, -f1-7 | cut -c1-200
done
if [ "${PMC:-0}" = "1" ]; then
  L=${LIBS%% *}
  for ctr in FETCH_SIZE WRITE_SIZE; do
    PROTO_LIB=$L timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/ppmc_${TAG}_$ctr -o run \
        -- python3 tools/protocol_pmc.py ${TAG}_$ctr > gpurun_out/ppmc_${TAG}_$ctr.log 2>&1
    rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/protocol_pmc_join.py gpurun_out/ppmc_${TAG}_FETCH_SIZE gpurun_out/ppmc_${TAG}_WRITE_SIZE \
      gpurun_out/protocol_ticks_${TAG}_FETCH_SIZE.json > gpurun_out/ppmc_${TAG}.json
  python3 -c "import json; d=json.load(open('gpurun_out/ppmc_${TAG}.json')); d.pop('per_tick'); print(json.dumps(d))"
fi
exit 0
