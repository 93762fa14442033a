// Type declarations of the brotli_amd Node drop-in: the public surface of countertype/brotli-lib
// (src/encode/encode.ts:22-27,50-90,290-409; src/decode/decode.ts:9-16,18-65;
// src/encode/enc-constants.ts:56-60), plus this engine's batch entry points.

export declare const EncoderMode: {
  readonly GENERIC: 0
  readonly TEXT: 1
  readonly FONT: 2
}
export type EncoderMode = (typeof EncoderMode)[keyof typeof EncoderMode]

export interface BrotliEncodeOptions {
  /** 0..11, default 11 (clamped) */
  quality?: number
  /** 10..24, default 22 (clamped) */
  lgwin?: number
  mode?: EncoderMode
  /** accepted, no effect (as in the reference) */
  sizeHint?: number
  /** extension: the encoder side of BrotliDecodeOptions.customDictionary; the stream decodes
   *  with (and only with) the same dictionary */
  customDictionary?: Uint8Array | Int8Array
}

export declare function brotliEncode(input: Uint8Array, options?: BrotliEncodeOptions): Uint8Array

export declare class BrotliEncoder {
  constructor(options?: BrotliEncodeOptions)
  /** the newly completed bytes (may be empty until enough input has arrived) */
  update(chunk: Uint8Array): Uint8Array
  finish(): Uint8Array
}

export interface BrotliDecodeOptions {
  maxOutputSize?: number
  /** compound dictionary (engine.ts:142-159) */
  customDictionary?: Uint8Array | Int8Array
}

/** options as a number: the legacy exact output size (truncate / zero-pad) */
export declare function brotliDecode(buffer: Uint8Array, options?: BrotliDecodeOptions | number): Uint8Array

/** decoded size from the first metablock header, -1 when unknown */
export declare function brotliDecodedSize(buffer: Uint8Array): number

export interface BatchOptions {
  /** shard the batch over this many GPUs (0: every visible one); absent: one GPU */
  gpus?: number
}
/** independent buffers in one GPU launch sequence (or one per GPU, options.gpus) */
export declare function brotliEncodeBatch(inputs: Uint8Array[], options?: BrotliEncodeOptions & BatchOptions): Uint8Array[]
export declare function brotliEncodeBatchAsync(inputs: Uint8Array[], options?: BrotliEncodeOptions & BatchOptions): Promise<Uint8Array[]>
/** a stream that fails to decode resolves to its Error in its slot */
export declare function brotliDecodeBatchAsync(inputs: Uint8Array[], options?: BatchOptions): Promise<(Uint8Array | Error)[]>
/** WOFF2 'glyf' transform (W3C WOFF2 section 5.1) of a TrueType font, on the GPU: FONT-mode input for brotliEncode */
export declare function woff2TransformGlyf(ttf: Uint8Array): Uint8Array
/** WOFF2 'hmtx' transform (section 5.4), or null when the table must stay untransformed */
export declare function woff2TransformHmtx(ttf: Uint8Array): Uint8Array | null
