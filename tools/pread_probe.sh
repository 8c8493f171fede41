set -e
F=${TMPDIR:-/tmp}/pp.bin
df -hT ${TMPDIR:-/tmp} > gpurun_out/pp_env.txt; taskset -p $$ >> gpurun_out/pp_env.txt; nproc >> gpurun_out/pp_env.txt
python3 -c "
import numpy as np
with open('$F','wb') as f:
    f.write(b'\0'*4096)
    a=np.arange(1<<27,dtype=np.uint64)
    for i in range(4): f.write(a.tobytes())
"
cat $F > /dev/null
timeout -k 10 120 paf-baseband2power_amd/bin/pread_probe $F 1073741824 > gpurun_out/pp_malloc.jsonl
timeout -k 10 120 paf-baseband2power_amd/bin/pread_probe $F 1073741824 shm > gpurun_out/pp_shm.jsonl
rm -f $F
