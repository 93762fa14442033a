# The working tree's library against libbrotli_amd_head.so (the last commit) on one box: the
# encoder's output digests of both (scripts/enc_digest.py: same bytes?), then exp_ab.sh's
# interleaved bench legs (WL, default "c2 c4"; R rounds)
cd $GRAFT_REPO_ROOT && OUT=gpurun_out/${TAG:-ab_digest} && mkdir -p $OUT && export TMPDIR=/tmp && \
BROTLI_AMD_LIB=$PWD/brotli-lib_amd/libbrotli_amd_head.so timeout -k 10 300 python3 scripts/enc_digest.py > $OUT/digest_head.json 2>$OUT/digest_head.err && \
timeout -k 10 300 python3 scripts/enc_digest.py > $OUT/digest_new.json 2>$OUT/digest_new.err && \
TAG=${TAG:-ab_digest} R=${R:-2} WL="${WL:-c2 c4}" bash scripts/exp_ab.sh
