cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_pipeline.py > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
for r in 1 2 3; do for v in s44 s48; do
 for c in euroc kitti; do
 ORBX_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --allow-diag --config $c --steps 100 --warmup 20 --cpu-sample 0 --no-latency --no-host-stream > /tmp/vb.log 2>&1 || { tail -5 /tmp/vb.log; exit 1; }
 python3 -c "import json;d=json.loads(open('/tmp/vb.log').read().strip().splitlines()[-1]);print('$v $c',d['value'],d['stage_ms_per_batch'])"
 done
done; done
