set -o pipefail
mkdir -p gpurun_out
d=$(mktemp -d)
timeout -k 5 60 tools/transport_big 1 $d > gpurun_out/r5g_big_r1.log 2>&1 &
p1=$!
timeout -k 5 60 tools/transport_big 0 $d > gpurun_out/r5g_big_r0.log 2>&1
rc0=$?
wait $p1
rc1=$?
echo "rc0=$rc0 rc1=$rc1"
cat gpurun_out/r5g_big_r0.log gpurun_out/r5g_big_r1.log | grep -v amdgpu.ids
