#!/usr/bin/env python3
"""Mechanical TypeScript type-erasure of the reference (countertype/brotli-lib) so its
own code can run on the container's Node v12 and act as the golden-vector generator.

TEST INFRASTRUCTURE ONLY.  Reads /root/reference (read-only), writes JavaScript into
oracle/_ref/ (git-ignored AND gpurun-ignored: the reference never travels, in any form).
Nothing in the product path imports or executes anything produced here.

Recipe: tokenize the TS, blank out type-only syntax (interfaces, type
aliases, `import type`, annotations, modifiers, `as T`, postfix `!`, generic parameter
lists), rewrite `const enum` to frozen objects and `a?.b` to a null-checked access,
resolve relative import specifiers to `.mjs`.  Two trees are produced:

  _ref/asis/   the reference exactly as shipped
  _ref/fixed/  the same plus the two one-line q10/q11 fixes the survey measured
               (Bug A backward-references-hq.ts:231-233, Bug B hash-binary-tree.ts:83-103)

Usage: python3 oracle/refgen/erase_ts.py [--ref /root/reference] [--out oracle/_ref]
"""
import argparse
import os
import re
import sys

PUNCT3 = ['>>>=', '===', '!==', '>>>', '<<=', '>>=', '**=', '...', '&&=', '||=', '??=']
PUNCT2 = ['=>', '==', '!=', '<=', '>=', '&&', '||', '??', '?.', '++', '--', '+=', '-=', '*=',
          '/=', '%=', '&=', '|=', '^=', '<<', '>>', '**']


class Tok:
    __slots__ = ('kind', 'text', 'ws')

    def __init__(self, kind, text, ws):
        self.kind = kind      # 'id', 'num', 'str', 'tpl', 'p' (punct), 'regex'
        self.text = text
        self.ws = ws          # whitespace/comments preceding the token (kept verbatim)

    def __repr__(self):
        return '%s:%r' % (self.kind, self.text)


def tokenize(src):
    toks = []
    i, n = 0, len(src)
    ws_start = 0
    prev_sig = None
    while True:
        # whitespace and comments
        while i < n:
            c = src[i]
            if c in ' \t\r\n':
                i += 1
            elif src.startswith('//', i):
                j = src.find('\n', i)
                i = n if j < 0 else j
            elif src.startswith('/*', i):
                j = src.find('*/', i + 2)
                i = n if j < 0 else j + 2
            else:
                break
        ws = src[ws_start:i]
        if i >= n:
            toks.append(Tok('eof', '', ws))
            break
        c = src[i]
        start = i
        if c.isalpha() or c in '_$':
            while i < n and (src[i].isalnum() or src[i] in '_$'):
                i += 1
            kind = 'id'
        elif c.isdigit() or (c == '.' and i + 1 < n and src[i + 1].isdigit()):
            while i < n and (src[i].isalnum() or src[i] in '._'):
                i += 1
            kind = 'num'
        elif c in '\'"':
            i += 1
            while src[i] != c:
                i += 2 if src[i] == '\\' else 1
            i += 1
            kind = 'str'
        elif c == '`':
            i += 1
            depth = 0
            while True:
                ch = src[i]
                if ch == '\\':
                    i += 2
                    continue
                if depth == 0 and ch == '`':
                    i += 1
                    break
                if src.startswith('${', i):
                    depth += 1
                    i += 2
                    continue
                if depth > 0 and ch == '}':
                    depth -= 1
                elif depth > 0 and ch == '{':
                    depth += 1
                i += 1
            kind = 'tpl'
        elif c == '/' and (prev_sig is None or (prev_sig.kind == 'p' and prev_sig.text not in (')', ']', '}'))
                           or (prev_sig.kind == 'id' and prev_sig.text in ('return', 'typeof'))):
            # regex literal (none in src, kept for safety)
            i += 1
            cls = False
            while True:
                ch = src[i]
                if ch == '\\':
                    i += 2
                    continue
                if ch == '[':
                    cls = True
                elif ch == ']':
                    cls = False
                elif ch == '/' and not cls:
                    i += 1
                    break
                i += 1
            while i < n and src[i].isalpha():
                i += 1
            kind = 'regex'
        else:
            kind = 'p'
            for cand in PUNCT3 + PUNCT2:
                if src.startswith(cand, i):
                    i += len(cand)
                    break
            else:
                i += 1
        t = Tok(kind, src[start:i], ws)
        toks.append(t)
        prev_sig = t
        ws_start = i
    return toks


OPEN = {'(': ')', '[': ']', '{': '}', '<': '>'}


def match_close(toks, i):
    """index of the token closing the bracket at toks[i]."""
    o = toks[i].text
    c = OPEN[o]
    depth = 0
    j = i
    while j < len(toks):
        t = toks[j].text
        if toks[j].kind == 'p':
            if o == '<':
                if t in ('<',):
                    depth += 1
                elif t in ('>',):
                    depth -= 1
                elif t == '>>':
                    depth -= 2
                elif t == '>>>':
                    depth -= 3
                elif t in ('(', '[', '{'):
                    j = match_close(toks, j)
                if depth <= 0:
                    return j
            else:
                if t == o:
                    depth += 1
                elif t == c:
                    depth -= 1
                    if depth == 0:
                        return j
        j += 1
    raise ValueError('unbalanced %s' % o)


def skip_type(toks, i):
    """toks[i] starts a type expression; return index just past it."""
    while True:
        t = toks[i]
        if t.kind == 'p' and t.text in ('{', '[', '('):
            j = match_close(toks, i) + 1
            if t.text == '(' and toks[j].text == '=>':
                i = skip_type(toks, j + 1)
            else:
                i = j
        elif t.kind == 'id' and t.text in ('typeof', 'keyof'):
            i += 1
            continue
        elif t.kind in ('id', 'str', 'num'):
            i += 1
            while toks[i].text == '.' and toks[i + 1].kind == 'id':
                i += 2
            if toks[i].text == '<':
                i = match_close(toks, i) + 1
        else:
            raise ValueError('cannot parse type at %r' % (toks[i:i + 5],))
        while toks[i].text == '[' and toks[i + 1].text == ']':
            i += 2
        if toks[i].text in ('|', '&'):
            i += 1
            continue
        return i


def blank(toks, a, b):
    """erase tokens [a, b) keeping newlines so line numbers survive."""
    for k in range(a, b):
        t = toks[k]
        nl = t.ws.count('\n') + t.text.count('\n')
        t.ws = '\n' * nl if nl else (' ' if t.ws else '')
        t.text = ''
        t.kind = 'gone'


def erase(src):
    toks = tokenize(src)
    N = len(toks)

    def nxt(i):
        i += 1
        while toks[i].kind == 'gone':
            i += 1
        return i

    def prv(i):
        i -= 1
        while i >= 0 and toks[i].kind == 'gone':
            i -= 1
        return i

    # pass 1: statements that vanish entirely, const enums
    i = 0
    while i < N:
        t = toks[i]
        if t.kind == 'id' and t.text == 'import' and toks[i + 1].text == 'type':
            j = i
            while toks[j].text != ';' and toks[j].kind != 'eof':
                if toks[j].text == '{':
                    j = match_close(toks, j)
                j += 1
                if toks[j].kind == 'str':
                    break
            blank(toks, i, j + 1 if toks[j].text != ';' else j + 1)
            i = j + 1
            continue
        if t.kind == 'id' and t.text == 'export' and toks[i + 1].text == 'type' and toks[i + 2].text == '{':
            j = match_close(toks, i + 2) + 1
            if toks[j].text == 'from':
                j += 2
            if toks[j].text == ';':
                j += 1
            blank(toks, i, j)
            i = j
            continue
        is_exp = t.text == 'export'
        k = i + 1 if is_exp else i
        if toks[k].kind == 'id' and toks[k].text == 'interface':
            j = k + 1
            while toks[j].text != '{':
                j += 1
            j = match_close(toks, j) + 1
            blank(toks, i, j)
            i = j
            continue
        if toks[k].kind == 'id' and toks[k].text == 'type' and toks[k + 1].kind == 'id' and toks[k + 2].text in ('=', '<'):
            j = k + 2
            if toks[j].text == '<':
                j = match_close(toks, j) + 1
            j = skip_type(toks, j + 1)
            if toks[j].text == ';':
                j += 1
            blank(toks, i, j)
            i = j
            continue
        if toks[k].text == 'const' and toks[k + 1].text == 'enum':
            # const enum E { A = 0, B } -> const E = Object.freeze({ A: 0, B: 1 })
            name = toks[k + 2].text
            ob = k + 3
            cb = match_close(toks, ob)
            toks[k + 1].text = ''
            toks[k + 2].text = name + ' ='
            toks[ob].text = 'Object.freeze({'
            toks[cb].text = '})'
            j = ob + 1
            val = -1
            while j < cb:
                if toks[j].kind == 'id':
                    if toks[j + 1].text == '=':
                        toks[j + 1].text = ':'
                        val = int(toks[j + 2].text, 0)
                        j += 3
                    else:
                        val += 1
                        toks[j].text = '%s: %d' % (toks[j].text, val)
                        j += 1
                else:
                    j += 1
            i = cb + 1
            continue
        i += 1

    # pass 2: annotations.  Find parameter lists and class bodies.
    class_bodies = set()
    i = 0
    while i < N:
        t = toks[i]
        if t.kind == 'id' and t.text == 'class':
            j = i + 1
            while toks[j].text != '{':
                j += 1
            class_bodies.add(j)
        i += 1

    enclosing = {}     # token index -> index of innermost enclosing '{'
    stack = []
    for i in range(N):
        enclosing[i] = stack[-1] if stack else None
        if toks[i].kind == 'p':
            if toks[i].text in ('{', '(', '['):
                stack.append(i if toks[i].text == '{' else -1)
            elif toks[i].text in ('}', ')', ']') and stack:
                stack.pop()
    param_lists = {}   # open-paren index -> True
    for i in range(N):
        t = toks[i]
        if t.kind != 'p' or t.text != '(':
            continue
        p = prv(i)
        pt = toks[p] if p >= 0 else None
        close = match_close(toks, i)
        after = nxt(close)
        is_params = False
        if pt is not None and pt.kind == 'id' and toks[prv(p)].text == 'function':
            is_params = True
        elif pt is not None and pt.text == 'function':
            is_params = True
        elif pt is not None and pt.text == '>' :
            # function name<T>(...)
            is_params = True
        elif toks[after].text == '=>':
            is_params = True
        elif toks[after].text == ':':
            # arrow with return type `(a: T): R =>`, or method signature
            try:
                e = skip_type(toks, after + 1)
                if toks[e].text in ('=>', '{'):
                    is_params = True
            except Exception:
                pass
        if not is_params and pt is not None and pt.kind == 'id' and enclosing.get(i) in class_bodies:
            # method / constructor in a class body: `name(` at body level followed by `{` or `:`
            if toks[after].text in ('{', ':'):
                if pt.text not in ('if', 'while', 'for', 'switch', 'catch', 'return', 'typeof'):
                    is_params = True
        if is_params:
            param_lists[i] = close

    def strip_in_params(o, c):
        j = o + 1
        depth = 0
        expect_name = True
        while j < c:
            t = toks[j]
            if t.kind == 'p' and t.text in ('(', '[', '{'):
                j = match_close(toks, j) + 1
                expect_name = False
                continue
            if t.kind == 'p' and t.text == ',':
                expect_name = True
                j += 1
                continue
            if t.kind == 'id' and t.text in ('private', 'public', 'protected', 'readonly') and toks[j + 1].kind == 'id':
                blank(toks, j, j + 1)
                j += 1
                continue
            if t.kind == 'p' and t.text == '?' and toks[j + 1].text == ':':
                blank(toks, j, j + 1)
                j += 1
                continue
            if t.kind == 'p' and t.text == ':':
                e = skip_type(toks, j + 1)
                blank(toks, j, e)
                j = e
                continue
            j += 1

    for o, c in param_lists.items():
        strip_in_params(o, c)
        a = nxt(c)
        if toks[a].text == ':':
            e = skip_type(toks, a + 1)
            blank(toks, a, e)
        # generic params before the paren: name<...>(
        p = prv(o)
        if p >= 0 and toks[p].text == '>':
            # find matching '<'
            depth = 0
            q = p
            while q >= 0:
                if toks[q].text == '>':
                    depth += 1
                elif toks[q].text == '<':
                    depth -= 1
                    if depth == 0:
                        break
                q -= 1
            blank(toks, q, p + 1)

    # variable declarations: let/const/var name: T
    for i in range(N):
        t = toks[i]
        if t.kind == 'id' and t.text in ('let', 'const', 'var'):
            j = nxt(i)
            if toks[j].kind == 'id':
                k = nxt(j)
                if toks[k].text == '!':
                    blank(toks, k, k + 1)
                    k = nxt(k)
                if toks[k].text == ':':
                    e = skip_type(toks, k + 1)
                    blank(toks, k, e)

    # class bodies: fields with modifiers / annotations
    for ob in class_bodies:
        cb = match_close(toks, ob)
        j = ob + 1
        at_member_start = True
        while j < cb:
            t = toks[j]
            if '\n' in t.ws:
                at_member_start = True
            if t.kind == 'p' and t.text in ('(', '[', '{'):
                j = match_close(toks, j) + 1
                at_member_start = toks[j - 1].text == '}'
                continue
            if at_member_start and t.kind == 'id' and t.text in ('private', 'public', 'protected', 'readonly', 'static') :
                if t.text != 'static':
                    blank(toks, j, j + 1)
                j += 1
                continue
            if at_member_start and t.kind == 'id':
                k = j + 1
                if toks[k].text in ('?', '!'):
                    blank(toks, k, k + 1)
                    k += 1
                if toks[k].text == ':':
                    e = skip_type(toks, k + 1)
                    blank(toks, k, e)
                    j = e
                    at_member_start = False
                    continue
            at_member_start = t.kind == 'p' and t.text in (';', '}')
            j += 1

    # `as Type` casts (not `import * as x`, not `{ a as b }` in import/export)
    i = 0
    while i < N:
        t = toks[i]
        if t.kind == 'id' and t.text == 'as':
            p = prv(i)
            if toks[p].text == '*':
                i += 1
                continue
            # inside import/export braces?
            q = p
            in_braces = False
            while q >= 0 and toks[q].text not in (';',):
                if toks[q].text in ('import', 'export'):
                    in_braces = True
                    break
                if toks[q].text in ('=', '(', 'return') or toks[q].text.startswith('\n'):
                    break
                q -= 1
            if in_braces:
                i += 1
                continue
            e = skip_type(toks, i + 1)
            blank(toks, i, e)
            i = e
            continue
        i += 1

    # postfix non-null assertion
    for i in range(1, N):
        t = toks[i]
        if t.kind == 'p' and t.text == '!':
            p = prv(i)
            if toks[p].kind in ('id', 'num') and toks[p].text not in ('return', 'typeof', 'case') or toks[p].text in (')', ']'):
                if toks[i + 1].text in ('.', '[', ')', ',', ';', ']') and t.ws == '':
                    blank(toks, i, i + 1)

    # generic args on `new X<T>(`
    for i in range(N):
        if toks[i].kind == 'id' and toks[i].text == 'new' and toks[i + 1].kind == 'id' and toks[i + 2].text == '<':
            c = match_close(toks, i + 2)
            blank(toks, i + 2, c + 1)

    # optional chaining a?.b  ->  (a == null ? undefined : a.b)
    for i in range(N):
        if toks[i].kind == 'p' and toks[i].text == '?.':
            p = prv(i)
            name = toks[p].text
            prop = toks[i + 1].text
            toks[p].text = '(%s == null ? undefined : %s.%s)' % (name, name, prop)
            toks[i].text = ''
            toks[i + 1].text = ''

    out = []
    for t in toks:
        out.append(t.ws)
        out.append(t.text)
    return ''.join(out)


IMPORT_RE = re.compile(r"""((?:import|export)\b[^;'"]*?from\s*|import\s*)(['"])(\.{1,2}/[^'"]+)\2""")


def fix_specifiers(js):
    def rep(m):
        spec = m.group(3)
        if not spec.endswith('.mjs'):
            spec = spec + '.mjs'
        return m.group(1) + m.group(2) + spec + m.group(2)
    return IMPORT_RE.sub(rep, js)


def drop_missing_named_imports(js_by_path):
    """TS elides imports of type-only names; drop specifiers the target does not export."""
    exports = {}
    for path, js in js_by_path.items():
        names = set(re.findall(r'export\s+(?:function|class|const|let|var)\s+([A-Za-z_$][\w$]*)', js))
        for grp in re.findall(r'export\s*\{([^}]*)\}', js):
            for part in grp.split(','):
                part = part.strip()
                if not part:
                    continue
                names.add(part.split(' as ')[-1].strip())
        exports[path] = names
    out = {}
    imp_re = re.compile(r"(import\s*\{)([^}]*)(\}\s*from\s*)(['\"])(\.{1,2}/[^'\"]+)\4")
    for path, js in js_by_path.items():
        def rep(m):
            target = os.path.normpath(os.path.join(os.path.dirname(path), m.group(5)))
            names = exports.get(target)
            if names is None:
                return m.group(0)
            keep = []
            for part in m.group(2).split(','):
                p = part.strip()
                if not p:
                    continue
                src_name = p.split(' as ')[0].strip()
                if src_name in names or src_name.startswith('*'):
                    keep.append(p)
            if not keep:
                return "import {} from %s%s%s" % (m.group(4), m.group(5), m.group(4))
            nl = m.group(2).count('\n')
            return m.group(1) + ' ' + ', '.join(keep) + ' ' + '\n' * nl + m.group(3) + m.group(4) + m.group(5) + m.group(4)
        out[path] = imp_re.sub(rep, js)
    return out


# The two one-line fixes, applied to the erased JS of _ref/fixed only.
FIXES = {
    'src/encode/backward-references-hq.mjs': [
        # Bug A: unused slots of the distance cache take the starting cache in order.
        ("  for (; idx < 4; idx++) {\n    distCache[idx] = startingDistCache[idx - (4 - idx)]\n  }",
         "  for (let k0 = idx; idx < 4; idx++) {\n    distCache[idx] = startingDistCache[idx - k0]\n  }"),
    ],
    'src/encode/hash-binary-tree.mjs': [
        # Bug B: an exhausted tree walk terminates the re-rooted tree (as upstream H10 does).
        ("        nodeRight = this.leftChildIndex(prevIx)\n        prevIx = this.forest[nodeRight]\n      }\n    }\n",
         "        nodeRight = this.leftChildIndex(prevIx)\n        prevIx = this.forest[nodeRight]\n      }\n"
         "      if (depthRemaining === 1 && shouldRerootTree) {\n"
         "        this.forest[nodeLeft] = this.invalidPos\n        this.forest[nodeRight] = this.invalidPos\n      }\n    }\n"),
    ],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/root/reference')
    ap.add_argument('--out', default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), '_ref'))
    args = ap.parse_args()
    files = {}
    for sub in ('src', 'test'):
        for root, _, names in os.walk(os.path.join(args.ref, sub)):
            for nm in names:
                if nm.endswith('.ts'):
                    full = os.path.join(root, nm)
                    rel = os.path.relpath(full, args.ref)
                    with open(full, encoding='utf-8') as f:
                        files[rel[:-3] + '.mjs'] = erase(f.read())
    files = {k: fix_specifiers(v) for k, v in files.items()}
    files = drop_missing_named_imports(files)
    prelude = ("if (typeof globalThis.atob === 'undefined') {\n"
               "  globalThis.atob = (s) => Buffer.from(s, 'base64').toString('binary')\n}\n")
    for variant in ('asis', 'fixed'):
        for rel, js in files.items():
            if variant == 'fixed':
                for a, b in FIXES.get(rel, []):
                    if a not in js:
                        sys.exit('fix anchor not found in %s' % rel)
                    js = js.replace(a, b)
            if rel.endswith('engine.mjs'):
                js = prelude + js
            if rel.startswith('test/'):
                js = js.replace("from 'vitest'", "from '../vitest_shim.mjs'")
            dst = os.path.join(args.out, variant, rel)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            with open(dst, 'w', encoding='utf-8') as f:
                f.write(js)
        shim = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'vitest_shim.mjs')
        with open(shim) as f, open(os.path.join(args.out, variant, 'vitest_shim.mjs'), 'w') as g:
            g.write(f.read())
        fx = os.path.join(args.out, variant, 'test', 'fixtures')
        if not os.path.exists(fx):
            os.symlink(os.path.join(args.ref, 'test', 'fixtures'), fx)
    print('erased %d files into %s/{asis,fixed}' % (len(files), args.out))


if __name__ == '__main__':
    main()
