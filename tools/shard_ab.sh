set -o pipefail
mkdir -p gpurun_out/shard_ab
for r in 1 2; do for v in s0 s1_gs192 s2_gs384; do
  AQ_LIB=$PWD/ppls_amd/_build/libaquad_$v.so timeout -k 10 120 python tools/try_shard.py --scale-k --k 16384 --reps 3 > gpurun_out/shard_ab/$v.$r.json 2> gpurun_out/shard_ab/$v.$r.err || { echo "$v failed"; tail -5 gpurun_out/shard_ab/$v.$r.err; exit 1; }
  echo "$r $v $(python -c "import json,sys; d=json.load(open('gpurun_out/shard_ab/$v.$r.json')); print({k: round(v['kernel_us']) for k, v in d.items() if k.startswith('shards')})")"
done; done
