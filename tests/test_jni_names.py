"""The JNI shim (jni/sparkbam_jni.c) and the Scala facades (jni/Native.scala,
jni/spark_bam_gpu.scala) name the reference's classes, constructors, imports and method
signatures; nothing here can compile them (no JVM in the image), so this pins every such name
against the reference's own declarations, recorded once by tools/gen_ref_api.py in
tests/golden/ref_scala_api.json (the shim threw a class that does not exist and
built case-class exceptions through a (String) constructor they do not have).

Checked:
  * every exception the shim throws: its class exists (the reference's declarations, the
    facades' own classes, or the JDK's), and the constructor descriptor the shim asks
    GetMethodID for is the JVM erasure of that class's real constructor;
  * every `Java_org_hammerlab_bam_gpu_Native_00024_<m>` export has an `@native def <m>` in
    object Native and vice versa;
  * every import from a reference package names a declaration of that package; every inline
    fully qualified reference name exists;
  * every construction / extractor use `X(...)` of a reference case class matches its
    constructor's arity (or an arity of its companion's apply);
  * every `override def` in a facade class overrides a method of that name and parameter
    lists in a reference (or facade) parent -- for GpuCanLoadBam the parameter names and
    types are the reference's exactly.
"""
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_ref_api  # noqa: E402  (the same declaration scanner the fixture was made with)

API = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_scala_api.json")))
REF = {}
for _d in API["declarations"]:
    REF.setdefault(_d["fqn"], []).append(_d)
SHIM = open(os.path.join(ROOT, "jni", "sparkbam_jni.c")).read()
FACADE_FILES = [os.path.join(ROOT, "jni", f) for f in ("Native.scala", "spark_bam_gpu.scala")]
FACADE_SRC = {f: open(f).read() for f in FACADE_FILES}
OURS = {}
for _f in FACADE_FILES:
    for _d in gen_ref_api.scan_file(_f, os.path.relpath(_f, ROOT)):
        OURS.setdefault(_d["fqn"], []).append(_d)

# packages whose declarations the fixture holds (the reference's own modules)
REF_PACKAGES = ("org.hammerlab.bam", "org.hammerlab.bgzf")
OUR_PACKAGE = "org.hammerlab.bam.gpu"
# third-party libraries the facades use; versions pinned by the reference's build.sbt (or
# its transitive dependencies, which it does not vendor): not checkable here
THIRD_PARTY = {
    "org.hammerlab.channel": "channel", "hammerlab.path": "paths", "hammerlab.iterator": "iterators",
    "org.hammerlab.hadoop": "spark_util", "org.hammerlab.genomics.loci": "loci", "org.hammerlab.spark": "spark_util",
    "htsjdk": None, "org.apache.spark": None, "scala": None, "java": None,
}
# JDK exceptions and the constructor descriptors the JDK gives them
JDK = {("java/io/IOException", "(Ljava/lang/String;)V"), ("java/io/EOFException", "(Ljava/lang/String;)V"),
       ("java/util/zip/DataFormatException", "(Ljava/lang/String;)V"),
       ("java/lang/IllegalArgumentException", "(Ljava/lang/String;)V"),
       ("java/lang/IllegalStateException", "(Ljava/lang/String;)V")}
PRIM = {"Int": "I", "Byte": "B", "Long": "J", "Short": "S", "Boolean": "Z", "Double": "D", "Float": "F",
        "Char": "C", "String": "Ljava/lang/String;"}


def value_class_erasure(name):
    """the JVM type a reference value class (extends AnyVal) erases to"""
    for fqn, ds in REF.items():
        if fqn.split(".")[-1] == name:
            for d in ds:
                if d["value_class"] and d["ctor"]:
                    return d["ctor"][0]["params"][0][1]
    return None


def descriptor(types):
    out = ""
    for t in types:
        t = t.strip()
        m = re.fullmatch(r"Array\[(\w+)\]", t)
        if m:
            out += "[" + PRIM[m.group(1)]
            continue
        t = value_class_erasure(t) or t
        if t in PRIM:
            out += PRIM[t]
        elif t == "Path":  # hammerlab.path.Path = org.hammerlab.paths.Path (paths 1.5.0)
            out += "Lorg/hammerlab/paths/Path;"
        else:
            out += "L" + t.replace(".", "/") + ";"
    return "(" + out + ")V"


def strip(src):
    return gen_ref_api.strip_comments(src)


def shim_exceptions():
    """(class, ctor descriptor) pairs the shim constructs"""
    defs = dict(re.findall(r'#define\s+(\w+)\s+"([^"]*)"', SHIM))
    table = re.search(r"EXCEPTIONS\[\]\s*=\s*\{(.*?)\n\};", SHIM, flags=re.S).group(1)
    pairs = set()
    for cls, ctor in re.findall(r"\{\s*SBH_E_\w+\s*,\s*([^,]+?)\s*,\s*([^}]+?)\s*\}", table):
        pairs.add((defs.get(cls, cls.strip('"')), defs.get(ctor, ctor.strip('"'))))
    for cls, ctor in re.findall(r'throw_new\(env,\s*("[^"]+"|\w+),\s*("[^"]+"|\w+)', SHIM):
        if cls in ("cls",):
            continue
        pairs.add((defs.get(cls, cls.strip('"')), defs.get(ctor, ctor.strip('"'))))
    other = re.search(r'OTHER_EXCEPTION\s*=\s*"([^"]+)"', SHIM).group(1)
    pairs.add((other, "(Ljava/lang/String;)V"))
    return pairs


def test_shim_exception_classes_and_constructors():
    pairs = shim_exceptions()
    assert ("org/hammerlab/bgzf/block/HeaderParseException", "(IBB)V") in pairs
    for cls, ctor in sorted(pairs):
        fqn = cls.replace("/", ".")
        if fqn.startswith("java."):
            assert (cls, ctor) in JDK, (cls, ctor)
            continue
        src = OURS if fqn.startswith(OUR_PACKAGE + ".") else REF
        ds = [d for d in src.get(fqn, []) if d["kind"] in ("class", "case class")]
        assert ds, f"{fqn}: no such class in the reference or the facades"
        ctors = [descriptor([t for _, t in d["ctor"][0]["params"]]) if d["ctor"] else "()V" for d in ds]
        assert ctor in ctors, (fqn, ctor, ctors)
        if src is REF:  # a reference exception: built from its own constructor, never (String)
            assert ctor != "(Ljava/lang/String;)V" or any(not d["ctor"] for d in ds), fqn


def test_shim_no_string_constructed_case_classes():
    """ThrowNew needs a (String) constructor, which the reference's case-class exceptions lack"""
    assert "ThrowNew" not in strip(SHIM)


def test_reference_exceptions_built_by_facade():
    """The two exceptions that need the file's Path are thrown by Native.rethrow with the
    reference's constructors (HeaderSearchFailedException.scala:7-12, FindRecordStart.scala:66-71)."""
    src = strip(FACADE_SRC[FACADE_FILES[0]])
    for name, arity in (("HeaderSearchFailedException", 3), ("NoReadFoundException", 3)):
        uses = re.findall(r"throw\s+" + name + r"\(", src)
        assert uses, name
    for fqn in ("org.hammerlab.bgzf.block.HeaderSearchFailedException", "org.hammerlab.bam.spark.NoReadFoundException"):
        assert fqn in REF


def test_native_methods_match_shim_exports():
    exports = set(re.findall(r"Java_org_hammerlab_bam_gpu_Native_00024_(\w+)\(", SHIM))
    native = set(re.findall(r"@native\s+def\s+(\w+)", strip(FACADE_SRC[FACADE_FILES[0]])))
    assert exports == native, (exports ^ native)


def imports(src):
    out = []
    for m in re.finditer(r"^\s*import\s+([\w.]+?)(?:\.\{([^}]*)\}|\.(\w+|_))\s*$", src, flags=re.M):
        pkg = m.group(1)
        names = [n.strip().split("⇒")[0].split("=>")[0].strip() for n in (m.group(2) or m.group(3)).split(",")]
        out += [(pkg, n) for n in names]
    return out


def is_ref_pkg(pkg):
    return pkg.startswith(REF_PACKAGES) and not pkg.startswith(OUR_PACKAGE)


def test_facade_imports_exist():
    for f, src in FACADE_SRC.items():
        for pkg, name in imports(strip(src)):
            if name == "_":
                continue
            if is_ref_pkg(pkg):
                fq = pkg + "." + name
                member = any(x["name"] == name for d in REF.get(pkg, []) for x in d["defs"])  # e.g. Checker.default
                assert fq in REF or member, f"{os.path.basename(f)}: import {fq}: not declared in the reference"
            elif pkg.startswith(OUR_PACKAGE):
                assert pkg + "." + name in OURS, f"{os.path.basename(f)}: import {pkg}.{name}: not a facade class"
            else:
                assert any(pkg == p or pkg.startswith(p + ".") for p in THIRD_PARTY), \
                    f"{os.path.basename(f)}: import from {pkg}: not the reference, the facades or a known dependency"
    # the pinned versions of the reference's own third-party libraries
    for lib in {v for v in THIRD_PARTY.values() if v}:
        assert lib in API["third_party_versions"], lib


def test_inline_qualified_names_exist():
    for f, src in FACADE_SRC.items():
        code = strip(src)
        code = re.sub(r"^\s*(import|package)\s+.*$", "", code, flags=re.M)
        for fq in set(re.findall(r"\b(org\.hammerlab\.(?:bam|bgzf)(?:\.\w+)+)", code)):
            if fq.startswith(OUR_PACKAGE):
                continue
            owner, name = fq.rsplit(".", 1)
            member = any(x["name"] == name for d in REF.get(owner, []) for x in d["defs"])
            assert fq in REF or member, f"{os.path.basename(f)}: {fq}"


def _visible_ref_classes(src):
    """simple name -> reference fqn, from the file's imports"""
    out = {}
    for pkg, name in imports(src):
        if is_ref_pkg(pkg) and name != "_" and pkg + "." + name in REF:
            out[name] = pkg + "." + name
    return out


def _args(src, i):
    """top-level argument count of the call whose '(' is at src[i]"""
    e = gen_ref_api.balanced(src, i, "(", ")")
    inner = src[i + 1:e - 1].strip()
    return 0 if not inner else len(gen_ref_api.split_top(inner))


def test_case_class_constructions_match_arity():
    checked = 0
    for f, src in FACADE_SRC.items():
        code = strip(src)
        vis = _visible_ref_classes(code)
        for name, fqn in vis.items():
            ds = REF[fqn]
            arities = set()
            for d in ds:
                if d["kind"] == "case class" and d["ctor"]:
                    arities.add(len(d["ctor"][0]["params"]))
                arities.update(d["apply_arities"])
            if not arities:
                continue
            for m in re.finditer(r"(?<![\w.])" + name + r"\(", code):
                prev = code[max(0, m.start() - 20):m.start()]
                if re.search(r"(class|trait|object|def|extends|with|new)\s+$", prev):
                    continue
                n = _args(code, m.end() - 1)
                assert n in arities, f"{os.path.basename(f)}: {name}(...) with {n} arguments; " \
                                     f"{fqn} takes {sorted(arities)}"
                checked += 1
    assert checked >= 10


# methods of JDK / Scala library parents the facades implement: name -> parameter-list shape
LIBRARY_METHODS = {"AutoCloseable": {"close": [0]}, "Closeable": {"close": [0]},
                   "Iterator": {"hasNext": [], "next": [0]}}


def _ref_parent_defs(parents, vis):
    defs = []
    for p in parents:
        for name, shape in LIBRARY_METHODS.get(p, {}).items():
            defs.append({"name": name, "params": [{"params": [None] * k} for k in shape]})
        for cand in (vis.get(p), OUR_PACKAGE + "." + p, p):
            for d in REF.get(cand, []) + OURS.get(cand, []):
                defs += d["defs"]
                defs += _ref_parent_defs(d["parents"], vis)
    return defs


def test_overrides_match_parent_signatures():
    checked = 0
    for f, src in FACADE_SRC.items():
        code = strip(src)
        vis = _visible_ref_classes(code)
        vis.update({"CanLoadBam": "org.hammerlab.bam.spark.load.CanLoadBam"})
        for fqn, ds in OURS.items():
            for d in ds:
                if d["file"] != os.path.relpath(f, ROOT):
                    continue
                mine = {x["name"]: x for x in d["defs"]}
                for name in re.findall(r"override\s+(?:protected\s+)?def\s+(\w+)",
                                       _body(code, fqn.split(".")[-1], d["kind"])):
                    m = mine[name]
                    cands = [x for x in _ref_parent_defs(d["parents"], vis) if x["name"] == name]
                    shape = [len(p["params"]) for p in m["params"]]
                    assert any([len(p["params"]) for p in c["params"]] == shape for c in cands), \
                        f"{fqn}.{name}{shape}: no parent method of that shape ({[c['params'] for c in cands]})"
                    checked += 1
    assert checked >= 10


def _body(code, simple, kind):
    kw = {"case class": r"case\s+class", "class": r"(?<!case )class", "trait": "trait",
          "object": r"(?<!package )object", "package object": r"package\s+object"}[kind]
    m = re.search(r"\b" + kw + r"\s+" + simple + r"\b", code)
    if not m:
        return ""
    i = code.find("{", m.end())
    body = code[i + 1:gen_ref_api.balanced(code, i, "{", "}") - 1]
    out, d = [], 0  # the body's own members only: nested blocks (method bodies, anonymous classes) blanked
    for ch in body:
        if ch == "{":
            d += 1
        elif ch == "}":
            d -= 1
        elif d == 0:
            out.append(ch)
    return "".join(out)


def test_gpu_can_load_bam_signatures_are_the_references():
    """GpuCanLoadBam overrides loadBam / loadSplitsAndReads / loadReadsAndPositions / loadReads /
    loadBamIntervals(path, LociSet, ...) with CanLoadBam's exact parameter names and types."""
    ref = {}
    for d in REF["org.hammerlab.bam.spark.load.CanLoadBam"]:
        for x in d["defs"]:
            ref.setdefault(x["name"], []).append(x["params"])
    ours = [d for d in OURS[OUR_PACKAGE + ".GpuCanLoadBam"]][0]["defs"]
    names = {x["name"] for x in ours}
    assert {"loadBam", "loadSplitsAndReads", "loadReadsAndPositions", "loadReads", "loadBamIntervals"} <= names
    for x in ours:
        assert x["params"] in ref[x["name"]], (x["name"], x["params"], ref[x["name"]])
