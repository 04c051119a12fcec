"""Resolve preprocessor conditionals on given macros in place (a small
unifdef: the image has none).  Used to delete measured-and-rejected compile
knobs from csrc/ (git history keeps the variants).

    python tools/unifdef.py -D PLVI_BF_NMS=0 -D PLVI_BF_LEAN=1 file...

A group (#if/#ifdef/#ifndef ... #elif ... #else ... #endif) is resolved when
every branch condition up to the taken one can be evaluated from the given
macros alone; other groups are kept verbatim (their bodies still processed).
The knob's own `#ifndef X / #define X v / #endif` default block is dropped,
and remaining uses of X in code are replaced by its value.
"""
import argparse
import re


def cond_value(expr, macros):
    """True/False if `expr` is decidable from `macros`, else None."""
    e = re.sub(r"//.*$", "", expr).strip()
    e = re.sub(r"/\*.*?\*/", "", e).strip()
    names = set(re.findall(r"\b[A-Za-z_]\w*\b", e)) - {"defined"}
    if not names or not names <= set(macros):
        return None
    py = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1", e)
    py = re.sub(r"defined\s+(\w+)", lambda m: "1", py)
    py = py.replace("&&", " and ").replace("||", " or ")
    py = re.sub(r"!(?!=)", " not ", py)
    for n in names:
        py = re.sub(r"\b%s\b" % n, "(%s)" % macros[n], py)
    return bool(eval(py))


def process(lines, macros):
    out = []
    # stack entries: [mode, taken, emitting_parent]; mode 'keep' = group kept
    # verbatim, 'resolve' = group being resolved
    stack = []
    emitting = True
    i = 0
    while i < len(lines):
        line = lines[i]
        m = re.match(r"^\s*#\s*(ifndef|ifdef|if|elif|else|endif)\b(.*)$", line)
        # drop `#ifndef X\n#define X v\n#endif` for a resolved knob
        if m and m.group(1) == "ifndef" and m.group(2).strip() in macros and i + 2 < len(lines) and \
                re.match(r"^\s*#\s*define\s+%s\b" % m.group(2).strip(), lines[i + 1]) and \
                re.match(r"^\s*#\s*endif", lines[i + 2]):
            i += 3
            continue
        if not m:
            if emitting:
                out.append(line)
            i += 1
            continue
        kw, rest = m.group(1), m.group(2)
        if kw in ("if", "ifdef", "ifndef"):
            if kw == "ifdef":
                n = rest.strip().split()[0]
                v = (n in macros) if n in macros else None
            elif kw == "ifndef":
                n = rest.strip().split()[0]
                v = (not (n in macros)) if n in macros else None
            else:
                v = cond_value(rest, macros)
            if v is None:
                stack.append(["keep", None, emitting])
                if emitting:
                    out.append(line)
            else:
                stack.append(["resolve", v, emitting])
                emitting = emitting and v
        elif kw == "elif":
            top = stack[-1]
            if top[0] == "keep":
                if top[2]:
                    out.append(line)
            else:
                if top[1]:
                    emitting = False
                else:
                    v = cond_value(rest, macros)
                    if v is None:
                        raise SystemExit("undecidable #elif after a resolved #if: " + line)
                    top[1] = v
                    emitting = top[2] and v
        elif kw == "else":
            top = stack[-1]
            if top[0] == "keep":
                if top[2]:
                    out.append(line)
            else:
                emitting = top[2] and not top[1]
                top[1] = True
        else:  # endif
            top = stack.pop()
            if top[0] == "keep":
                if top[2]:
                    out.append(line)
            emitting = top[2]
        i += 1
    assert not stack, "unbalanced conditionals"
    text = "".join(out)
    for n, v in macros.items():
        text = re.sub(r"\b%s\b" % n, str(v), text)
    return text


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("files", nargs="+")
    a = ap.parse_args()
    macros = {}
    for d in a.D:
        k, _, v = d.partition("=")
        macros[k] = v or "1"
    for f in a.files:
        src = open(f).read().splitlines(keepends=True)
        new = process(src, macros)
        if new != "".join(src):
            open(f, "w").write(new)
            print("updated", f)


if __name__ == "__main__":
    main()
