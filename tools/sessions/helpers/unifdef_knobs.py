#!/usr/bin/env python3
"""Resolve compile-time A/B knobs to their default values in place (a small
partial `unifdef`): each `#ifndef K / #define K v / #endif` default block of a
listed knob is removed, and every `#if / #elif` whose expression uses only
listed knobs and integer literals is evaluated and its dead arms dropped.
Conditionals on anything else (UWVK_STAMPS, PSP_SIDE, ...) are kept as they
are, with the knob conditionals nested inside them still resolved.  Plain C++
uses of a knob outside directives are reported, not rewritten.

usage: tools/unifdef_knobs.py FILE... --knobs K1,K2,...  (defaults read from FILES)
"""
import re
import sys

DEF_RE = re.compile(r"^\s*#\s*ifndef\s+(\w+)\s*(//.*)?$")


def collect_defaults(lines, knobs):
    vals = {}
    for i, ln in enumerate(lines):
        m = DEF_RE.match(ln)
        if m and m.group(1) in knobs and i + 1 < len(lines):
            d = re.match(r"^\s*#\s*define\s+(\w+)\s+(.*?)\s*(//.*)?$", lines[i + 1])
            if d and d.group(1) == m.group(1):
                vals[m.group(1)] = d.group(2)
    return vals


def strip_default_blocks(lines, knobs):
    out, i = [], 0
    while i < len(lines):
        m = DEF_RE.match(lines[i])
        d = re.match(r"^\s*#\s*define\s+(\w+)", lines[i + 1]) if m and i + 1 < len(lines) else None
        if m and m.group(1) in knobs and d and d.group(1) == m.group(1):
            # #ifndef K ... #endif (the #define plus continuation comment lines)
            j = i + 1
            while not re.match(r"^\s*#\s*endif", lines[j]):
                j += 1
            i = j + 1
            continue
        out.append(lines[i])
        i += 1
    return out


def c_eval(expr, vals):
    e = re.sub(r"//.*$", "", expr)
    e = re.sub(r"/\*.*?\*/", "", e).strip()
    ids = set(re.findall(r"[A-Za-z_]\w*", e)) - {"defined"}
    if not ids or not ids <= set(vals):
        return None
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if m.group(1) in vals else "0", e)
    for _ in range(6):  # defaults may refer to other knobs
        e = re.sub(r"\b([A-Za-z_]\w*)\b", lambda m: "(%s)" % vals[m.group(1)] if m.group(1) in vals else m.group(1), e)
    py = e.replace("&&", " and ").replace("||", " or ")
    py = re.sub(r"!(?!=)", " not ", py)
    try:
        return int(bool(eval(py, {}, {})))
    except Exception:
        return None


def resolve(lines, vals):
    out = []
    # stack entries: [kind, state] kind 'k' (knob-resolved) or 'x' (kept);
    # for 'k': state = (taken_any, emitting)
    stack = []

    def emitting():
        return all(s[1] for s in stack if s[0] == "k")

    for ln in lines:
        m = re.match(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$", ln)
        if not m:
            if emitting():
                out.append(ln)
            continue
        kw, rest = m.group(1), m.group(2)
        if kw in ("if", "ifdef", "ifndef"):
            expr = rest
            if kw == "ifdef":
                expr = "defined(%s)" % rest.split()[0]
            elif kw == "ifndef":
                expr = "!defined(%s)" % rest.split()[0]
            v = c_eval(expr, vals) if (kw == "if" or rest.split()[0] in vals) else None
            if v is None:
                stack.append(["x", True, False])
                if emitting():
                    out.append(ln)
            else:
                stack.append(["k", bool(v), bool(v)])
        elif kw == "elif":
            top = stack[-1]
            if top[0] == "x":
                v = c_eval(rest, vals)
                if v is not None and emitting():
                    # a kept #if with a resolvable #elif: keep the directive structure
                    out.append(re.sub(r"#\s*elif.*", "#elif %d" % v, ln))
                elif emitting():
                    out.append(ln)
            else:
                v = c_eval(rest, vals)
                if v is None:
                    raise SystemExit("unresolvable #elif inside a knob conditional: " + ln)
                taken = top[2]
                top[1] = (not taken) and bool(v)
                top[2] = taken or bool(v)
        elif kw == "else":
            top = stack[-1]
            if top[0] == "x":
                if emitting():
                    out.append(ln)
            else:
                top[1] = not top[2]
                top[2] = True
        else:  # endif
            top = stack.pop()
            if top[0] == "x" and emitting():
                out.append(ln)
    assert not stack, "unbalanced conditionals"
    return out


def main():
    args = sys.argv[1:]
    i = args.index("--knobs")
    knobs = set(args[i + 1].split(","))
    files = args[:i] + args[i + 2:]
    vals = {}
    texts = {}
    for f in files:
        texts[f] = open(f).read().split("\n")
        vals.update(collect_defaults(texts[f], knobs))
    missing = knobs - set(vals)
    if missing:
        raise SystemExit("no default found for: %s" % ", ".join(sorted(missing)))
    print("defaults:", vals)
    for f, lines in texts.items():
        lines = strip_default_blocks(lines, knobs)
        lines = resolve(lines, vals)
        open(f, "w").write("\n".join(lines))
        for n, ln in enumerate(lines, 1):
            for k in knobs:
                if re.search(r"\b%s\b" % k, ln):
                    print("%s:%d: %s" % (f, n, ln.strip()))


if __name__ == "__main__":
    main()
