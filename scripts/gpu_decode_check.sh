set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'brotli-lib_amd/python'); sys.path.insert(0,'tests')
import brotli_amd, _oracle
d = open('tests/golden/vectors/x.compressed','rb').read()
print('x ->', brotli_amd.brotliDecode(d))
d = open('tests/golden/vectors/alice29.txt.compressed','rb').read()
o = brotli_amd.brotliDecode(d); print('alice ok', o == open('tests/golden/vectors/alice29.txt','rb').read())
" > gpurun_out/first.log 2>&1 && \
timeout -k 10 900 python3 -m pytest tests/test_gpu_decode.py -x -q > gpurun_out/gpu_decode.log 2>&1
echo "exit=$?"
