"""Summarise scripts/exp_ab.sh output: per workload and library, value / encode / decode MB/s."""
import glob
import json
import os
import sys
d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, '*_*.json'))):
    rows = [json.loads(l) for l in open(f) if l.startswith('{')]
    if not rows:
        continue
    def col(k):
        return [r.get(k) for r in rows]
    print('%-24s value %s  enc %s  dec %s  ratio %s' % (os.path.basename(f), col('value'), col('encode_MBps'),
                                                        col('decode_MBps'), sorted(set(col('compressed_ratio')))))
