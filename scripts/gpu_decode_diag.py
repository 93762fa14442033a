"""Run the decode error corpus case by case on the GPU, logging progress (diagnostics)."""
import base64, hashlib, json, os, sys, time
sys.path.insert(0, 'brotli-lib_amd/python'); sys.path.insert(0, 'tests')
import brotli_amd, _oracle
g = json.load(open('tests/golden/decode_errors.json'))['cases']
log = open('gpurun_out/diag.log', 'w')
bad = 0
for i, c in enumerate(g):
    data = base64.b64decode(c['in_b64'])
    exp = _oracle.decode(data)
    exp = ('Brotli error code: %d' % exp) if isinstance(exp, int) else hashlib.sha256(exp).hexdigest()
    log.write('%d len=%d ... ' % (i, len(data))); log.flush()
    t = time.time()
    try:
        got = hashlib.sha256(brotli_amd.brotliDecode(data)).hexdigest()
    except brotli_amd.BrotliError as e:
        got = str(e)
    ok = got == exp
    bad += not ok
    log.write('%s %.3fs %s\n' % ('ok' if ok else 'MISMATCH got=%s exp=%s b64=%s' % (got, exp, c['in_b64']), time.time() - t, '')); log.flush()
log.write('bad=%d\n' % bad)
