"""Print the headline fields of bench JSON lines side by side (A/B runs under gpurun_out/)."""
import json
import sys

KEYS = ['dp_parse', 'dp_sample', 'find_matches', 'decode_streams_kernel', 'decode_parts_kernel', 'emit', 'huffman', 'codes']
for p in sys.argv[1:]:
    try:
        d = json.load(open(p))
    except Exception as e:
        print(p, 'unreadable', e)
        continue
    r = d.get('ratio_same_sample') or {}
    k = d.get('kernel_ms_per_step', {})
    print('%-34s MB/s %8.1f enc %8.1f dec %8.1f ratio %.5f vs_native %s | %s' % (
        p.split('gpurun_out/')[-1], d['value'], d.get('encode_MBps', 0), d.get('decode_MBps', 0),
        d.get('compressed_ratio', 0), r.get('gpu_vs_node_native'),
        ' '.join('%s=%.1f' % (x, k[x]) for x in KEYS if x in k)))
