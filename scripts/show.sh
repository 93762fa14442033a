# print the results of the last gpurun iteration
tail -2 gpurun_out/iter_tests.log
grep -v amdgpu.ids gpurun_out/dectime.log 2>/dev/null | tail -2
python3 -c "
import json;d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]);print(d['value'],'enc',d['encode_MBps'],'dec',d['decode_MBps'],'ratio',d['compressed_ratio']);print(d['kernel_ms_per_step'])"
