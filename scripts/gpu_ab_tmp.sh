cd /root/repo; mkdir -p gpurun_out/ab2; export TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab2/$tag.json 2> gpurun_out/ab2/$tag.err || { echo "$tag failed"; tail -3 gpurun_out/ab2/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab2/$tag.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('$tag', d['value'], d['ms_per_step'], {k: round(s.get(k,0),2) for k in ('seeds','descent_tile','crop_cc','output','size_filter','smooth_seeds')})"; }
for s in 2 3 4 6; do run c3_s$s python3 -u bench.py --streams $s --steps 8 --warmup 2 --no-cpu-baseline --no-host --no-e2e; done
