"""Generate tests/golden/ref_scala_api.json: the reference's Scala declarations the JNI shim
(jni/sparkbam_jni.c) and the Scala facades (jni/Native.scala) name.

Run once here, where /root/reference exists (it is read as text only; nothing of it is
compiled or run):

    python tools/gen_ref_api.py /root/reference > tests/golden/ref_scala_api.json

For every class / case class / trait / object declared under */src/main/scala the file records
its fully qualified name, kind, constructor parameter lists (name, declared type), whether it
is a value class (extends AnyVal: its JVM erasure is the single parameter's type), the arities
of its companion's `apply` methods, and the `def`s it declares (name, parameter lists) -- the
data tests/test_jni_names.py checks the shim's class names / constructor signatures and the
facades' imports, constructions and overrides against.  Third-party libraries the reference
depends on (build.sbt) are listed with their pinned versions; their classes cannot be checked
here.
"""
import json
import os
import re
import sys

KW = re.compile(r"\b(case\s+class|class|trait|object)\s+([A-Za-z_][A-Za-z0-9_]*)")


def strip_comments(s):
    s = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), s, flags=re.S)
    s = re.sub(r"//[^\n]*", "", s)
    # string literals: keep the quotes, drop the contents (braces inside strings)
    s = re.sub(r'"""(.*?)"""', '""', s, flags=re.S)
    s = re.sub(r'"(\\.|[^"\\\n])*"', '""', s)
    s = re.sub(r"'(\\.|[^'\\\n])'", "' '", s)
    return s


def balanced(s, i, o, c):
    """index just past the bracket group opening at s[i] == o"""
    d = 0
    j = i
    while j < len(s):
        if s[j] == o:
            d += 1
        elif s[j] == c:
            d -= 1
            if d == 0:
                return j + 1
        j += 1
    return len(s)


def split_top(s, sep=","):
    out, d, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            d += 1
        elif ch in ")]}":
            d -= 1
        if ch == sep and d == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [x.strip() for x in out]


def params(group):
    """'(a: Int, b: Byte = 1)' -> [['a', 'Int'], ['b', 'Byte']]; implicit lists marked"""
    inner = group[1:-1].strip()
    implicit = inner.startswith("implicit")
    if implicit:
        inner = inner[len("implicit"):]
    out = []
    for p in split_top(inner):
        p = re.sub(r"^(@\S+\s+)*(override\s+)?(private\s+|protected\s+)?(val|var)?\s*", "", p.strip())
        if ":" not in p:
            continue
        name, typ = p.split(":", 1)
        typ = typ.split("=")[0].strip()
        out.append([name.strip(), re.sub(r"\s+", " ", typ)])
    return {"implicit": implicit, "params": out}


def scan_file(path, rel):
    src = strip_comments(open(path, encoding="utf-8").read())
    pkg = []
    for m in re.finditer(r"^\s*package\s+([\w.]+)\s*$", src, flags=re.M):
        pkg.append(m.group(1))
    package = ".".join(pkg)
    decls = []
    # brace-depth map: owner stack of (depth, fqn)
    stack = []
    depth = 0
    i = 0
    pending = None  # a declaration whose body '{' is still to come
    while i < len(src):
        m = KW.match(src, i)
        if m and (i == 0 or not (src[i - 1].isalnum() or src[i - 1] == "_")):
            kind = re.sub(r"\s+", " ", m.group(1))
            name = m.group(2)
            owner = decls[stack[-1][1]]["fqn"] if stack and stack[-1][1] >= 0 else (
                "<def>" if stack else None)
            if name == "object" or owner == "<def>":
                i = m.end()
                continue
            fqn = (owner + "." if owner else (package + "." if package else "")) + name
            if kind == "object" and src[max(0, i - 8):i].strip().endswith("package"):
                kind = "package object"
            j = m.end()
            while j < len(src) and src[j] in " \t":
                j += 1
            if j < len(src) and src[j] == "[":
                j = balanced(src, j, "[", "]")
            plists = []
            while True:
                k = j
                while k < len(src) and src[k] in " \t\n":
                    k += 1
                # `private` / annotations before a constructor list
                mm = re.match(r"(private|protected)(\[[\w.]+\])?\s*", src[k:])
                if mm:
                    k += mm.end()
                if k < len(src) and src[k] == "(":
                    e = balanced(src, k, "(", ")")
                    plists.append(params(src[k:e]))
                    j = e
                else:
                    break
            head_end = j
            # header up to the body or the end of the declaration
            n = j
            d2 = 0
            while n < len(src):
                ch = src[n]
                if ch in "([":
                    d2 += 1
                elif ch in ")]":
                    d2 -= 1
                elif d2 == 0 and ch == "{":
                    break
                elif d2 == 0 and ch == "\n":
                    # a declaration without a body ends at a line that starts a new statement
                    rest = src[n + 1:].lstrip(" \t")
                    if not re.match(r"(extends|with|\)|\{)", rest):
                        break
                n += 1
            header = src[head_end:n]
            value_class = bool(re.search(r"\bextends\s+AnyVal\b", header))
            parents = re.findall(r"\b(?:extends|with)\s+([\w.]+)", header)
            decls.append({"fqn": fqn, "kind": kind, "file": rel, "ctor": plists, "value_class": value_class,
                          "parents": parents, "defs": [], "apply_arities": []})
            if n < len(src) and src[n] == "{":
                pending = len(decls) - 1
            i = n
            continue
        ch = src[i]
        if ch == "{":
            depth += 1
            if pending is not None:
                stack.append((depth, pending))
                pending = None
            elif stack and stack[-1][0] == depth - 1 and re.search(r"\bdef\b[^{}]*$", src[max(0, i - 400):i]):
                stack.append((depth, -1))  # a method body: nothing declared in it is recorded
        elif ch == "}":
            if stack and stack[-1][0] == depth:
                stack.pop()
            depth -= 1
        elif src.startswith("def ", i) and (i == 0 or not src[i - 1].isalnum()) and stack \
                and stack[-1][0] == depth and stack[-1][1] >= 0:
            mm = re.match(r"def\s+([^\s(\[:=]+)", src[i:])
            if mm:
                j = i + mm.end()
                if j < len(src) and src[j] == "[":
                    j = balanced(src, j, "[", "]")
                pl = []
                while j < len(src) and src[j] in " \t\n(":
                    if src[j] == "(":
                        e = balanced(src, j, "(", ")")
                        pl.append(params(src[j:e]))
                        j = e
                    else:
                        j += 1
                dcl = decls[stack[-1][1]]
                dcl["defs"].append({"name": mm.group(1), "params": pl})
                if mm.group(1) == "apply":
                    dcl["apply_arities"].append(len(pl[0]["params"]) if pl else 0)
                i = j
                continue
        i += 1
    return decls


def third_party(root):
    txt = open(os.path.join(root, "build.sbt"), encoding="utf-8").read()
    return {k.replace(" ", ""): v for k, v in re.findall(r"([\w.]+)\s*→\s*\"([^\"]+)\"", txt)}


def main(root):
    decls = []
    for d, _, files in os.walk(root):
        if "/src/main/scala" not in d.replace(os.sep, "/") + "/":
            continue
        for f in sorted(files):
            if f.endswith(".scala"):
                p = os.path.join(d, f)
                decls += scan_file(p, os.path.relpath(p, root))
    decls.sort(key=lambda x: (x["fqn"], x["kind"]))
    json.dump({"generated_by": "tools/gen_ref_api.py", "third_party_versions": third_party(root),
               "declarations": decls}, sys.stdout, indent=1, sort_keys=True)
    sys.stdout.write("\n")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
