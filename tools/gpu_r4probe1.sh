set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/r4probe1; mkdir -p $D
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_df1.json 2> $D/bench_df1.err &&
timeout -k 10 300 python -u tools/driver_form_probe.py > $D/probe.jsonl 2> $D/probe.err &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $D/bench_df2.json 2> $D/bench_df2.err
echo "exit=$?"
