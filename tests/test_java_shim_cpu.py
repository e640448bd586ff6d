"""The Java drop-in builds for the reference's toolchain: Java 8 (/root/reference/pom.xml:50, the
Flink 1.8 connector's JVM).  No JDK exists in this container, so:

* the main source set (java/main) is checked for every construct newer than Java 8 by pattern -- records, pattern
  instanceof, switch rules / multi-label cases, var, collection factories (List/Set/Map.of), StackWalker, the Java 16
  absolute bulk ByteBuffer.put, text blocks, Java 9+ String / Stream methods, java.lang.foreign;
* the FFM binding lives only in the optional java/ffm source set (JDK 22+);
* the JNI binding (java/jni/scotty_jni.c, the default) is compiled with gcc -fsyntax-only -Wall -Werror against
  include/scotty_mi355x.h and the type-check stub tests/jni_stub/jni.h, and every `native` method of JniApi.java has
  its JNIEXPORT symbol there.
CPU only."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAIN = os.path.join(ROOT, "java", "main", "de", "tub", "dima", "scotty", "slicing")
FFM = os.path.join(ROOT, "java", "ffm", "de", "tub", "dima", "scotty", "slicing")
JNI_C = os.path.join(ROOT, "java", "jni", "scotty_jni.c")

NEWER_THAN_8 = [
    (r"\brecord\s+\w+\s*[(<]", "record class (Java 16)"),
    (r"\binstanceof\s+[\w.]+(?:<[^>]*>)?\s+[a-z]\w*\b", "pattern-matching instanceof (Java 16)"),
    (r"\bcase\b[^:;\n]*->", "switch rule (Java 14)"),
    (r"\bcase\s+[\w.]+\s*,", "multi-label case (Java 14)"),
    (r"=\s*switch\s*\(|return\s+switch\s*\(", "switch expression (Java 14)"),
    (r"\byield\b", "yield (Java 14)"),
    (r"(?<![\w.])var\s+\w+\s*[=:]", "local variable type inference (Java 10)"),
    (r"\b(?:List|Set|Map)\.(?:of|copyOf|ofEntries)\s*\(", "collection factory (Java 9/10)"),
    (r"\bStackWalker\b", "StackWalker (Java 9)"),
    (r"\.put\(\s*\d+\s*,\s*\w+\s*,", "absolute bulk ByteBuffer.put (Java 16)"),
    (r"\.get\(\s*\d+\s*,\s*\w+\s*,\s*\d+\s*,", "absolute bulk ByteBuffer.get (Java 13)"),
    (r'"""', "text block (Java 15)"),
    (r"\.(?:isBlank|strip|stripLeading|stripTrailing|lines|repeat|formatted|indent)\(", "String method (Java 11+)"),
    (r"\.toList\(\)", "Stream.toList (Java 16)"),
    (r"\.orElseThrow\(\)", "Optional.orElseThrow() (Java 10)"),
    (r"java\.lang\.foreign", "FFM API (Java 22)"),
    (r"new\s+\w+(?:\.\w+)*\s*<>\s*\([^)]*\)\s*\{", "anonymous class with diamond (Java 9)"),
    (r"\btry\s*\(\s*\w+\s*\)", "try-with-resources on an effectively final variable (Java 9)"),
    (r"\bsealed\b|\bpermits\b|\bnon-sealed\b", "sealed classes (Java 17)"),
    (r"\.takeWhile\(|\.dropWhile\(|\.iterate\([^)]*,[^)]*,", "Stream method (Java 9)"),
    (r"\bProcessHandle\b|\bHttpClient\b|\bCleaner\b", "JDK 9+ API"),
]


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", lambda m: " " * len(m.group(0)), src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _strip_strings(src):
    return re.sub(r'"(?:\\.|[^"\\\n])*"', '""', src)


def _main_sources():
    return sorted(os.path.join(MAIN, f) for f in os.listdir(MAIN) if f.endswith(".java"))


def test_main_source_set_is_java8():
    files = _main_sources()
    assert len(files) == 7, files
    bad = []
    for f in files:
        raw = _strip_comments(open(f).read())
        for pat, what in NEWER_THAN_8:
            src = raw if pat == '"""' else _strip_strings(raw)  # class names in string literals are not code
            for m in re.finditer(pat, src):
                line = src[:m.start()].count("\n") + 1
                bad.append("%s:%d %s: %r" % (os.path.basename(f), line, what, m.group(0)))
    assert not bad, "\n".join(bad)


def test_patterns_catch_the_constructs_they_name():
    """The checker itself: each pattern fires on a sample of its construct and not on its Java 8 spelling."""
    newer = ["record Row(long a) {}", "if (w instanceof TumblingWindow t) {", "case COUNT -> 1;",
             "case A, B:", "return switch (op) {", "var x = 1;", "Set.of(\"a\")", "StackWalker.getInstance()",
             "ts.put(0, tsBuf, 0, n);", "java.lang.foreign.Linker", "s.isBlank()"]
    java8 = ["final class Row {", "if (w instanceof TumblingWindow) {", "case COUNT:", "switch (op) {",
             "int x = 1;", "Collections.singleton(\"a\")", "Thread.currentThread().getStackTrace()",
             "ts.putLong(8, t);", "to.put(from);", "s.isEmpty()"]
    for src in newer:
        assert any(re.search(p, src) for p, _ in NEWER_THAN_8), src
    for src in java8:
        assert not any(re.search(p, src) for p, _ in NEWER_THAN_8), src


def test_ffm_binding_only_in_optional_source_set():
    assert os.listdir(FFM) == ["FfmApi.java"]
    for f in _main_sources():
        assert "FfmApi" not in _strip_comments(open(f).read()).replace('"de.tub.dima.scotty.slicing.FfmApi"', ""), f
    # JNI is the default binding; FFM only on request
    api = open(os.path.join(MAIN, "NativeApi.java")).read()
    assert 'System.getProperty("scotty.native.binding", "jni")' in api


def test_keyed_engine_has_explicit_opt_in():
    """An explicit opt-in (factory, thread scope, system property, extra caller names) beside the connector-name
    fallback, which searches the whole stack (no fixed frame limit)."""
    op = open(os.path.join(MAIN, "SlicingWindowOperator.java")).read()
    ke = open(os.path.join(MAIN, "KeyedEngine.java")).read()
    assert "public static <T> SlicingWindowOperator<T> perKey(" in op
    assert "public static KeyedScope keyedScope()" in op
    assert '"scotty.keyed.engine"' in ke and '"scotty.keyed.callers"' in ke
    assert "getStackTrace()" in ke and "limit(" not in _strip_comments(ke)
    # the connector-name search runs once per call site and thread, not once per key (1 M keys): the class context
    # (no StackTraceElements) and the frame that matched last time
    assert "getClassContext()" in ke and "LAST_HIT" in ke


GENERIC_DECL = re.compile(r"\b(?:List|Set|Map|Collection|Iterable|ThreadLocal)\s*<((?:[^<>]|<[^<>]*>)*)>\s+\w+\s*=\s*"
                          r"new\s+\w+\s*<((?:[^<>]|<[^<>]*>)*)>\s*\(")


def _norm(t):
    return re.sub(r"\s+", "", t)


def test_generic_instantiations_match_their_declarations():
    """javac type-checks what this container cannot: a declaration `List<A> x = new ArrayList<B>(...)` with B != A is
    an incompatible-types error on every JDK (round 4's Java 8 rewrite of the diamonds produced three).  Every such
    declaration in the main source set must instantiate exactly its declared type arguments (or a diamond)."""
    bad, seen = [], 0
    for f in _main_sources():
        src = _strip_strings(_strip_comments(open(f).read()))
        for m in GENERIC_DECL.finditer(src):
            seen += 1
            decl, inst = _norm(m.group(1)), _norm(m.group(2))
            if inst and inst != decl:
                line = src[:m.start()].count("\n") + 1
                bad.append("%s:%d declared <%s>, instantiated <%s>" % (os.path.basename(f), line, decl, inst))
    assert seen >= 8, seen
    assert not bad, "\n".join(bad)


def test_generic_check_catches_a_mismatch():
    src = "private final List<NativeFunctions.Binding> b = new ArrayList<AggregateWindow>();"
    m = GENERIC_DECL.search(src)
    assert m and _norm(m.group(1)) != _norm(m.group(2))
    ok = "Map<Integer, List<Row>> pending = new HashMap<Integer, List<Row>>();"
    m = GENERIC_DECL.search(ok)
    assert m and _norm(m.group(1)) == _norm(m.group(2))


def _javac():
    import shutil
    j = shutil.which("javac")
    if j:
        return j
    home = os.environ.get("JAVA_HOME")
    if home and os.path.exists(os.path.join(home, "bin", "javac")):
        return os.path.join(home, "bin", "javac")
    return None


def test_main_source_set_compiles_with_javac_when_a_jdk_exists(tmp_path):
    """The real check where a JDK exists: javac -source 8 over java/main against stubs of the reference's core API
    types the shim imports would be needed, so only the syntax/type pass of the shim's own classes runs
    (-proc:none, -implicit:none, the reference jars on SCOTTY_REF_CLASSPATH).  Skipped without a JDK -- this
    container and the GPU box have none; the pattern checks above stand in for it."""
    javac = _javac()
    cp = os.environ.get("SCOTTY_REF_CLASSPATH")
    if not javac or not cp:
        pytest.skip("no JDK / reference classpath here (javac %s, SCOTTY_REF_CLASSPATH %s)" % (javac, cp))
    r = subprocess.run([javac, "-source", "8", "-target", "8", "-proc:none", "-implicit:none", "-d", str(tmp_path),
                        "-cp", cp] + _main_sources(), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_jni_binding_compiles_against_the_header():
    cmd = ["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
           "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"), JNI_C]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_native_method_has_its_jni_symbol():
    java = _strip_comments(open(os.path.join(MAIN, "JniApi.java")).read())
    natives = re.findall(r"\bnative\s+[\w\[\]]+\s+(\w+)\s*\(", java)
    assert len(natives) == 10, natives
    c = open(JNI_C).read()
    exported = set(re.findall(r"JNIEXPORT\s+\w+\s+JNICALL\s+(Java_\w+)\s*\(", c))
    want = {"Java_de_tub_dima_scotty_slicing_JniApi_" + n.replace("_", "_1") for n in natives}
    assert want == exported, (want ^ exported)
