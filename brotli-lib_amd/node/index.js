'use strict'
// brotli_amd for Node: the public surface of countertype/brotli-lib (package.json:7-23)
// over the MI355X engine.  Argument handling and error messages follow the reference:
//   brotliEncode(input, {quality, lgwin, mode, sizeHint})    src/encode/encode.ts:50-90
//   new BrotliEncoder(options).update(chunk) / .finish()     src/encode/encode.ts:290-409
//   brotliDecode(data, {maxOutputSize, customDictionary} | outputSize)
//                                                            src/decode/decode.ts:18-65
//   brotliDecodedSize(data)                                  src/decode/decode.ts:9-11
//   EncoderMode                                              src/encode/enc-constants.ts:56-60
// The addon (brotli_amd.node) is built by __graft_entry__.build(); there is no JavaScript
// fallback, a missing GPU throws.
const path = require('path')
const native = require(path.join(__dirname, 'brotli_amd.node'))

const EncoderMode = Object.freeze({ GENERIC: 0, TEXT: 1, FONT: 2 })

function clampOptions(options) {
  const o = options || {}
  let quality = 11
  let lgwin = 22
  let mode = EncoderMode.GENERIC
  if (o.quality !== undefined) quality = Math.max(0, Math.min(11, o.quality))
  if (o.lgwin !== undefined) lgwin = Math.max(10, Math.min(24, o.lgwin))
  if (o.mode !== undefined) mode = o.mode
  return [quality | 0, lgwin | 0, mode | 0]
}

// customDictionary (extension, the encoder side of brotliDecode's option): Uint8Array / Int8Array
function dictOf(options) {
  const d = options && options.customDictionary
  if (!d) return null
  return d instanceof Uint8Array ? d : new Uint8Array(d.buffer, d.byteOffset, d.byteLength)
}

function toU8(b) {
  return new Uint8Array(b.buffer, b.byteOffset, b.byteLength)
}

function brotliEncode(input, options) {
  const [q, lg, m] = clampOptions(options)
  return toU8(native.encode(input, q, lg, m, dictOf(options)))
}

class BrotliEncoder {
  constructor(options) {
    const [q, lg, m] = clampOptions(options)
    // options.streamChunk (extension): throughput mode, see brotli_amd.h mib_enc_opts.stream_chunk
    const sc = options && options.streamChunk ? Math.max(0, options.streamChunk) : 0
    this._h = native.encoderNew(q, lg, m, dictOf(options), sc)
  }
  update(input) {
    return toU8(native.encoderUpdate(this._h, input))
  }
  finish() {
    return toU8(native.encoderFinish(this._h))
  }
}

function brotliDecodedSize(buffer) {
  return native.decodedSize(buffer)
}

function brotliDecode(buffer, options) {
  let exact = -1
  let maxOutputSize
  let dict = null
  if (typeof options === 'number') {
    exact = options
  } else if (options) {
    maxOutputSize = options.maxOutputSize
    const d = options.customDictionary
    if (d) dict = d instanceof Uint8Array ? d : new Uint8Array(d.buffer, d.byteOffset, d.byteLength)
  }
  try {
    return toU8(native.decode(buffer, maxOutputSize === undefined ? -1 : maxOutputSize, exact, dict))
  } catch (e) {
    if (e && e.size !== undefined) throw new Error(`Decompressed size ${e.size} exceeds limit ${maxOutputSize}`)
    throw e
  }
}

// options.gpus: shard the batch over that many GPUs (0: every visible one); absent: one GPU
function gpusOf(options) {
  const g = options && options.gpus
  return g === undefined || g === null ? -1 : Math.max(0, g | 0)
}

// batch entry point of this engine: independent buffers in one GPU launch sequence
function brotliEncodeBatch(inputs, options) {
  const [q, lg, m] = clampOptions(options)
  return native.encodeBatch(inputs, q, lg, m, gpusOf(options), dictOf(options)).map(toU8)
}

// the same, off the JS thread: the GPU work runs on a worker (napi_async_work), a Promise
// resolves to the outputs (decode: a stream that fails gives its Error in its slot)
function brotliEncodeBatchAsync(inputs, options) {
  const [q, lg, m] = clampOptions(options)
  return native.encodeBatchAsync(inputs, q, lg, m, gpusOf(options), dictOf(options)).then((outs) => outs.map(toU8))
}
function brotliDecodeBatchAsync(inputs, options) {
  return native.decodeBatchAsync(inputs, gpusOf(options)).then((outs) => outs.map((o) => (o instanceof Error ? o : toU8(o))))
}

// the FONT-mode caller's step before brotliEncode (reference README.md:63): the WOFF2
// transformed 'glyf' / 'hmtx' tables of a TrueType font, computed on the GPU
function woff2TransformGlyf(ttf) {
  return toU8(native.woff2Glyf(ttf))
}
function woff2TransformHmtx(ttf) {
  const r = native.woff2Hmtx(ttf)
  return r === null ? null : toU8(r)
}

module.exports = {
  brotliEncode, BrotliEncoder, brotliDecode, brotliDecodedSize, EncoderMode,
  brotliEncodeBatch, brotliEncodeBatchAsync, brotliDecodeBatchAsync,
  woff2TransformGlyf, woff2TransformHmtx,
}
