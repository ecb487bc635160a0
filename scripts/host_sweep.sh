# host-path pipeline knobs, alternating configurations in one call (box noise)
set -e
for pass in 1 2; do
  for cfg in "16777216 1 0" "16777216 1 1" "8388608 1 1" "4194304 1 1"; do
    set -- $cfg
    if [ $2 = 1 ]; then export PM_HOST_DIRECT=1; else unset PM_HOST_DIRECT; fi
    if [ $3 = 1 ]; then export PM_HOST_DIRECT_IN=1; else unset PM_HOST_DIRECT_IN; fi
    PM_PIPE_POSITIONS=$1 timeout -k 10 300 python scripts/host_path_rate.py > gpurun_out/hr.json 2>/dev/null
    echo "$pass $1 $2 $3 $(python -c "import json;r=json.load(open('gpurun_out/hr.json'));print(r['rt_read_block_gid_GBps'],r['rt_read_block_ids_GBps'],r['ac_read_block_gid_GBps'])")" >> gpurun_out/hr_sweep.txt
  done
done
