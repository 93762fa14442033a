// placeholder: the GPU encoder lands in the next commit
#include <hip/hip_runtime.h>
#include "common.h"
extern "C" void mib_encode_ws_free(void *ws) {}
extern "C" int mib_encode(const uint8_t *in, size_t n, const mib_enc_opts *o, mib_buf *out) { return MIB_E_INVALID_ARG; }
extern "C" int mib_encode_batch(const mib_span *in, size_t k, const mib_enc_opts *o, mib_buf *out, int *status) { return MIB_E_INVALID_ARG; }
extern "C" int mib_ctx_encode(mib_ctx *c, const mib_enc_opts *o, const uint8_t *d_in, const uint64_t *in_offsets,
                   size_t k, uint8_t *d_out, uint64_t out_cap, uint64_t *out_offsets, void *stream) { return MIB_E_INVALID_ARG; }
extern "C" mib_encoder *mib_encoder_new(const mib_enc_opts *o) { return nullptr; }
extern "C" int mib_encoder_update(mib_encoder *e, const uint8_t *in, size_t n, mib_buf *out) { return MIB_E_INVALID_ARG; }
extern "C" int mib_encoder_finish(mib_encoder *e, mib_buf *out) { return MIB_E_INVALID_ARG; }
extern "C" void mib_encoder_free(mib_encoder *e) {}
