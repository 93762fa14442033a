"""Oracle analysis (CPU): the reference's q11 parse restated (oracle_encode.c) with only the N longest matches per position kept (oracle_set_keep_matches); prints compressed/input per setting (profiles/r06/oracle_kept_matches.txt)."""
import sys, os, ctypes
from concurrent.futures import ProcessPoolExecutor
sys.path.insert(0,'/root/repo/tests'); sys.path.insert(0,'/root/repo/brotli-lib_amd/python'); sys.path.insert(0,'/root/repo/tests/golden/woff2')
import _oracle
from brotli_amd import datagen
def job(a):
    kind, seed, keep = a
    if kind=='c4': d = datagen.enwik_text(1<<18, seed)
    else:
        import make_golden
        d = datagen.glyf_font_stream(1<<18, seed, transform=make_golden.transform)
    lib=_oracle.lib(); lib.oracle_set_keep_matches(ctypes.c_uint(keep))
    return len(_oracle.encode(d, 11, 22, 2 if kind=='c3' else 0)), len(d)
with ProcessPoolExecutor(8) as ex:
  for kind in ['c4','c3']:
    for keep in [0,8,6,4]:
      r=list(ex.map(job,[(kind,s,keep) for s in range(1000,1004)]))
      print(kind,keep,sum(a for a,b in r)/sum(b for a,b in r),flush=True)
