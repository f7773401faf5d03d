# attention overlap: bit-identity test, kernel-pair probe, then headline contract off / on
export TMPDIR=/tmp; O=gpurun_out/overlap; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "overlap or layer_executor" > $O/test.log 2>&1; e=$?; tail -1 $O/test.log; [ $e -eq 0 ] || exit $e
timeout -k 10 400 python3 tools/overlap_probe.py > $O/probe.txt 2>&1; e=$?; grep -v amdgpu.ids $O/probe.txt | tail -7; [ $e -eq 0 ] || exit $e
for v in 0 1; do
  timeout -k 10 450 env K8SRCA_ATTN_OVERLAP=$v python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-hints-steps 0 > $O/bench$v.log 2>&1; e=$?
  grep '^{' $O/bench$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; print('overlap', $v, d['value'], d['p50_latency_s'], 'ctx Mtok/s', round(e['decode_ctx_tokens']/(d['ms_per_step']*d['steps']/1000)/1e6,2), 'prefill tok/s', d['throughput']['prefill_tok_per_s'])"
  [ $e -eq 0 ] || exit $e
done
