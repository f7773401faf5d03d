# in-kernel split-KV merge: bit-identity test, decode probe off/on, concurrency-1 latency off/on, headline on
export TMPDIR=/tmp; O=gpurun_out/merge; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "merge or paged_decode" > $O/test.log 2>&1; e=$?; tail -1 $O/test.log; [ $e -eq 0 ] || exit $e
for v in 0 1; do
  timeout -k 10 200 env K8SRCA_DECODE_MERGE=$v python3 tools/decode_probe.py > $O/probe$v.txt 2>&1 || { tail -3 $O/probe$v.txt; exit 1; }
  grep "scattered part=None" $O/probe$v.txt | sed "s/^/merge=$v /"
done
for v in 0 1; do
  timeout -k 10 300 env K8SRCA_DECODE_MERGE=$v python3 bench.py --incidents 1 --quantum 1 --steps 10 --warmup 2 --no-hints-steps 0 > $O/c1_$v.json 2> $O/c1_$v.err || { tail -3 $O/c1_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c1_$v.json').read().strip().splitlines()[-1]); print('c1 merge=$v', d['value'], d['p50_latency_s'], d['work_per_analysis'])"
done
timeout -k 10 450 env K8SRCA_DECODE_MERGE=1 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-hints-steps 0 > $O/bench1.log 2>&1; e=$?
grep '^{' $O/bench1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine']; print('headline merge=1', d['value'], d['p50_latency_s'], 'ctx Mtok/s', round(e['decode_ctx_tokens']/(d['ms_per_step']*d['steps']/1000)/1e6,2))"
exit $e
