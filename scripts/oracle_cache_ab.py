"""Oracle analysis (CPU): the reference's q11 parse restated (oracle_encode.c) with only some of the 16 distance-cache candidates (oracle_set_cache_mask); prints compressed/input per setting (profiles/r06/oracle_cache_candidates.txt)."""
import sys, os, ctypes, time
from concurrent.futures import ProcessPoolExecutor
sys.path.insert(0,'/root/repo/tests'); sys.path.insert(0,'/root/repo/brotli-lib_amd/python'); sys.path.insert(0,'/root/repo/tests/golden/woff2')
import _oracle
from brotli_amd import datagen
def job(a):
    kind, seed, mask = a
    if kind=='c4': d = datagen.enwik_text(1<<18, seed)
    else:
        import make_golden
        d = datagen.glyf_font_stream(1<<18, seed, transform=make_golden.transform)
    lib=_oracle.lib(); lib.oracle_set_cache_mask(ctypes.c_uint(mask))
    mode = 2 if kind=='c3' else 0
    return len(_oracle.encode(d, 11, 22, mode)), len(d)
masks={'all':0xFFFF,'none':0,'j0':1,'j0-3':0xF}
with ProcessPoolExecutor(8) as ex:
  for kind in ['c4','c3']:
    for name,m in masks.items():
      r=list(ex.map(job,[(kind,s,m) for s in range(1000,1004)]))
      print(kind,name,sum(a for a,b in r)/sum(b for a,b in r),flush=True)
