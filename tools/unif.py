"""Resolve conditional-compilation blocks of known macros in place (a minimal unifdef):
python tools/unif.py FILE NAME=VALUE ... (NAME=- : undefined). Handles #if NAME, #if !NAME,
#if NAME == N / != N, #ifdef / #ifndef NAME, #else, #endif; a "#ifndef NAME / #define NAME v /
#endif" default block is dropped. Blocks of other macros are kept as they are. Used in round 6
to take the measured-loser A/B branches out of the product kernels (the removal is kept as a
patch under profiles/r06/)."""
import re
import sys


def cond_value(line, known):
    s = line.strip()
    m = re.match(r"#\s*ifdef\s+(\w+)", s)
    if m and m.group(1) in known:
        return known[m.group(1)] is not None
    m = re.match(r"#\s*ifndef\s+(\w+)", s)
    if m and m.group(1) in known:
        return known[m.group(1)] is None
    m = re.match(r"#\s*if\s+(!?)\s*(\w+)\s*(?:(==|!=)\s*(\d+))?\s*(?://.*)?$", s)
    if m and m.group(2) in known:
        v = known[m.group(2)]
        v = 0 if v is None else int(v)
        if m.group(3) == "==":
            r = v == int(m.group(4))
        elif m.group(3) == "!=":
            r = v != int(m.group(4))
        else:
            r = v != 0
        return (not r) if m.group(1) else r
    return None


def main():
    path = sys.argv[1]
    known = {}
    for kv in sys.argv[2:]:
        k, v = kv.split("=")
        known[k] = None if v == "-" else v
    lines = open(path).read().split("\n")
    out = []
    stack = []  # (resolved: bool or None, taking: bool)
    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        # default block: #ifndef NAME / #define NAME ... / #endif
        m = re.match(r"#\s*ifndef\s+(\w+)", s)
        if m and m.group(1) in known and i + 2 < len(lines) and re.match(r"#\s*define\s+" + m.group(1) + r"\b", lines[i + 1].strip()) \
                and lines[i + 2].strip().startswith("#endif") and known[m.group(1)] is not None:
            i += 3
            continue
        active = all(t for _, t in stack)
        if re.match(r"#\s*if", s):
            cv = cond_value(ln, known)
            if cv is None:
                stack.append((None, True))
                if active:
                    out.append(ln)
            else:
                stack.append((True, cv))
            i += 1
            continue
        if re.match(r"#\s*else", s):
            res, take = stack[-1]
            if res is None:
                if all(t for _, t in stack[:-1]):
                    out.append(ln)
            else:
                stack[-1] = (True, not take)
            i += 1
            continue
        if re.match(r"#\s*endif", s):
            res, _ = stack.pop()
            if res is None and all(t for _, t in stack):
                out.append(ln)
            i += 1
            continue
        if active:
            out.append(ln)
        i += 1
    assert not stack, "unbalanced"
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
