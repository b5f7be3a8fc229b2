"""Extract the plain-SQL plan-shape test cases from the reference's ScalaTest sources.

Only ``test("name", "sql" + "sql" ..., <numDruidQueries>, ...)`` calls whose SQL is made of plain
string literals are taken (DSL-interpolated ``date"..."`` (triple-quoted) cases are skipped).  Used by
tests/test_reference_corpus.py; reads the read-only reference checkout when it is mounted."""
import os
import re

REF_TESTS = "/root/reference/src/test/scala/org/sparklinedata/druid/client/test"

_CALL = re.compile(r'\b(test|cTest)\(\s*"([^"]+)"\s*,')


def _string_concat(src, i):
    """Parse `"..." + "..." + ...` (plain or triple-quoted, optional .stripMargin) starting at i."""
    out = []
    n = len(src)
    while True:
        while i < n and src[i] in " \t\r\n":
            i += 1
        if src.startswith('"""', i):
            j = src.index('"""', i + 3)
            s = src[i + 3:j]
            i = j + 3
            if src.startswith(".stripMargin", i):
                s = "\n".join(re.sub(r"^\s*\|", "", ln) for ln in s.split("\n"))
                i += len(".stripMargin")
            out.append(s)
        elif i < n and src[i] == '"':
            j = i + 1
            buf = []
            while src[j] != '"':
                if src[j] == "\\":
                    buf.append(src[j + 1])
                    j += 2
                    continue
                buf.append(src[j])
                j += 1
            out.append("".join(buf))
            i = j + 1
        else:
            return None, i
        while i < n and src[i] in " \t\r\n":
            i += 1
        if i < n and src[i] == "+":
            i += 1
            continue
        return "".join(out), i


def cases():
    if not os.path.isdir(REF_TESTS):
        return []
    out = []
    for fn in sorted(os.listdir(REF_TESTS)):
        if not fn.endswith(".scala"):
            continue
        src = open(os.path.join(REF_TESTS, fn)).read()
        for m in _CALL.finditer(src):
            kind, name = m.group(1), m.group(2)
            sql, i = _string_concat(src, m.end())
            if not sql or "$" in sql:
                continue
            rest = src[i:i + 40]
            if kind == "test":
                mm = re.match(r"\s*,\s*(\d+)", rest)
                if not mm:
                    continue
                out.append((fn[:-6], name, "shape", " ".join(sql.split()), int(mm.group(1)), None))
            else:
                mm = re.match(r"\s*,\s*", rest)
                sql2, _ = _string_concat(src, i + mm.end()) if mm else (None, 0)
                if sql2 and "$" not in sql2:
                    out.append((fn[:-6], name, "ctest", " ".join(sql.split()), None, " ".join(sql2.split())))
    return out


if __name__ == "__main__":
    cs = cases()
    print(len(cs))
    for c in cs[:5]:
        print(c)
