// Minimal stand-in for the three vitest entry points the reference's test file uses
// (describe / it / expect).  TEST INFRASTRUCTURE ONLY: lets the type-erased reference
// run its own test/brotli.test.ts on Node 12 to validate the erasure (oracle/refgen).
const tests = []
let prefix = []
export function describe(name, fn) { prefix.push(name); fn(); prefix.pop() }
export function it(name, fn) { tests.push([prefix.concat(name).join(' > '), fn]) }
function eq(a, b) {
  if (a === b) return true
  if (a && b && typeof a === 'object' && typeof b === 'object') {
    if (a.length !== b.length) return false
    const ka = Object.keys(a), kb = Object.keys(b)
    if (ka.length !== kb.length) return false
    for (const k of ka) if (!eq(a[k], b[k])) return false
    return true
  }
  return false
}
export function expect(v) {
  const m = {
    toBe(x) { if (v !== x) throw new Error(`expected ${x} got ${v}`) },
    toEqual(x) { if (!eq(v, x)) throw new Error('toEqual mismatch') },
    toBeGreaterThan(x) { if (!(v > x)) throw new Error(`expected > ${x} got ${v}`) },
    toBeLessThan(x) { if (!(v < x)) throw new Error(`expected < ${x} got ${v}`) },
    toThrow(re) {
      let threw = false
      try { v() } catch (e) { threw = true; if (re && !String(e.message).match(re)) throw new Error('wrong error ' + e.message) }
      if (!threw) throw new Error('expected throw')
    },
  }
  return m
}
export async function run() {
  let pass = 0, fail = 0
  for (const [name, fn] of tests) {
    try { await fn(); pass++ } catch (e) { fail++; console.log('FAIL', name, '-', e.message) }
  }
  console.log(`pass=${pass} fail=${fail}`)
  return fail
}
