set -o pipefail
cd /root/repo; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/convbench.py --blocks --variants 13 --mb 1024 --iters 10 --ablate 0 512 --shapes l3.c2+id l4.c2+id > gpurun_out/r03_ab1_id.log 2>&1 || exit $?
cat gpurun_out/r03_ab1_id.log
bash tools/ab_env.sh "tree:SAD_HALO256=0 tree:SAD_HALO256=1" 3 2>&1 | tee gpurun_out/r03_ab1_bf16.log || exit 1
for i in 1 2; do for h in 0 1; do
  r=$(SAD_HALO256=$h timeout -k 10 200 python bench.py --dtype bf16x3 --kernels-only --steps 8 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["backbone"]["ms_per_step"])') || exit 1
  echo "x3 HALO256=$h: $r" | tee -a gpurun_out/r03_ab1_x3.log
done; done
