# Print the results of tools/gpu/run_ab_quick.sh
O=${1:-gpurun_out/ab}
tail -1 $O/tests.log
for w in 8 4 2; do echo "s$w $(python -c "import json;print(json.load(open('$O/s$w.json'))['fps'])" 2>&1 | tail -1)"; done
python -c "import json;d=json.load(open('$O/full.json'));print('full', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], 'hash', d['hash']['frames_per_s'], d['hash']['kernel_avg_us'])"
