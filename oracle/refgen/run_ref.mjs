// TEST INFRASTRUCTURE ONLY: run the type-erased reference (oracle/_ref/<variant>) on a batch
// of jobs and record what it returns.  Used by make_goldens.py; never shipped, never on the GPU box.
// usage: node run_ref.mjs <jobs.json> <results.json>
import { readFileSync, writeFileSync } from 'fs'
import * as zlib from 'zlib'
import { createHash } from 'crypto'
import { dirname, join } from 'path'
import { fileURLToPath } from 'url'
const here = dirname(fileURLToPath(import.meta.url))
const jobs = JSON.parse(readFileSync(process.argv[2], 'utf8'))
const mods = {}
async function lib(variant) {
  if (!mods[variant]) {
    const root = join(here, '..', '_ref', variant, 'src')
    mods[variant] = {
      enc: await import(join(root, 'encode', 'encode.mjs')),
      dec: await import(join(root, 'decode', 'decode.mjs')),
      bt: await import(join(root, 'encode', 'hash-binary-tree.mjs')),
    }
  }
  return mods[variant]
}
const sha = (b) => createHash('sha256').update(b).digest('hex')
async function main() {
const results = []
for (const job of jobs) {
  const m = await lib(job.variant || 'fixed')
  const input = job.in_b64 !== undefined ? Buffer.from(job.in_b64, 'base64') : readFileSync(job.in)
  const r = { id: job.id }
  try {
    if (job.op === 'encode') {
      const t0 = process.hrtime.bigint()
      const out = m.enc.brotliEncode(new Uint8Array(input), job.opts || {})
      r.ms = Number(process.hrtime.bigint() - t0) / 1e6
      r.len = out.length
      r.sha256 = sha(out)
      if (out.length <= (job.inline_max || 4096)) r.out_b64 = Buffer.from(out).toString('base64')
      try { r.native_roundtrip = Buffer.compare(zlib.brotliDecompressSync(Buffer.from(out)), input) === 0 } catch (e) { r.native_roundtrip = false }
    } else if (job.op === 'decode') {
      let opts = job.opts
      if (job.dict_b64 !== undefined) {   // customDictionary (compound dictionary), as Uint8Array or Int8Array
        const d = Buffer.from(job.dict_b64, 'base64')
        const u = new Uint8Array(d.length)
        u.set(d)
        opts = Object.assign({}, opts || {}, { customDictionary: job.dict_int8 ? new Int8Array(u.buffer) : u })
      }
      const out = m.dec.brotliDecode(new Uint8Array(input), opts)
      r.len = out.length
      r.sha256 = sha(out)
    } else if (job.op === 'bt_matches') {
      // per-position match lists as createHqZopfliBackwardReferences pass 1 collects them
      const h = m.bt.createBinaryTreeHasher(job.lgwin || 22, input.length)
      const lists = []
      const maxBack = (1 << (job.lgwin || 22)) - 16
      for (let i = 0; i + 3 < input.length; i++) {
        const ms = h.findAllMatches(input, (1 << (job.lgwin || 22)) - 1, i, input.length - i, Math.min(i, maxBack))
        if (ms.length > 0 && ms[ms.length - 1].length > 325) {
          lists.push([i, [[ms[ms.length - 1].distance, ms[ms.length - 1].length]]])
          i += ms[ms.length - 1].length - 1
          continue
        }
        lists.push([i, ms.map((x) => [x.distance, x.length])])
      }
      r.lists = lists
    }
  } catch (e) {
    r.error = String(e.message)
  }
  results.push(r)
}
writeFileSync(process.argv[3], JSON.stringify(results))
}
main().catch((e) => { console.error(e); process.exit(1) })
