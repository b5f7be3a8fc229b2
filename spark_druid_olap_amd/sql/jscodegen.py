"""Render SQL expressions as Druid JavaScript function text.

The reference compiles un-pushable single-dimension predicates/groupings and multi-metric aggregate
expressions to Rhino JavaScript (``sd/jscodegen/JSCodeGenerator.scala:76-451``,
``sd/jscodegen/JSAggGenerator.scala:34-161``).  On MI355X the JavaScript is *not* what executes:
single-dimension expressions are evaluated over the dictionary (``sql/functions.py``) and metric
expressions run in the scan kernel's expression VM.  The text is still generated so QuerySpecs keep
the reference's JSON shape (EXPLAIN DRUID REWRITE, query history, ``EXECUTE QUERY`` round trips);
aggregator bodies use the arithmetic subset the VM accepts (``query/jsfunc.jsagg_to_expr``).
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional

from . import ast as A
from .functions import typeof


class JSGenError(ValueError):
    pass


_CMP = {"=": "==", "<>": "!=", "<": "<", "<=": "<=", ">": ">", ">=": ">="}
_ARITH = {"+", "-", "*", "/", "%"}


def js_expr(e: A.Expr, names: Dict[int, str]) -> str:
    """JS source for an expression; ``names`` maps attribute ids to JS variable names."""
    if isinstance(e, A.Ref):
        if e.rid not in names:
            raise JSGenError(f"unbound {e.sql()}")
        return names[e.rid]
    if isinstance(e, A.Lit):
        if e.value is None:
            return "null"
        if isinstance(e.value, bool):
            return "true" if e.value else "false"
        if isinstance(e.value, (int, float)):
            return repr(e.value)
        return json.dumps(str(e.value))
    if isinstance(e, A.BinOp):
        l, r = js_expr(e.l, names), js_expr(e.r, names)
        if e.op in _ARITH:
            return f"({l} {e.op} {r})"
        if e.op in _CMP:
            return f"({l} {_CMP[e.op]} {r})"
        if e.op == "and":
            return f"({l} && {r})"
        if e.op == "or":
            return f"({l} || {r})"
        raise JSGenError(e.op)
    if isinstance(e, A.UnOp):
        c = js_expr(e.child, names)
        return f"(!{c})" if e.op == "not" else f"(-{c})"
    if isinstance(e, A.Cast):
        c = js_expr(e.child, names)
        if e.to in ("double", "float") or e.to.startswith("decimal"):
            return f"Number({c})"
        if e.to in ("int", "bigint", "smallint", "tinyint"):
            return f"Math.floor(Number({c}))"
        if e.to == "string":
            return f"String({c})"
        return c
    if isinstance(e, A.IsNull):
        c = js_expr(e.child, names)
        return f"({c} {'!=' if e.negated else '=='} null)"
    if isinstance(e, A.InList):
        c = js_expr(e.child, names)
        vals = ", ".join(js_expr(i, names) for i in e.items)
        s = f"([{vals}].indexOf({c}) >= 0)"
        return f"(!{s})" if e.negated else s
    if isinstance(e, A.Case):
        out = js_expr(e.else_, names) if e.else_ is not None else "null"
        for c, v in reversed(e.whens):
            out = f"(({js_expr(c, names)}) ? ({js_expr(v, names)}) : ({out}))"
        return out
    if isinstance(e, A.Call):
        a = [js_expr(x, names) for x in e.args]
        n = e.name
        if n in ("upper", "ucase"):
            return f"({a[0]}).toUpperCase()"
        if n in ("lower", "lcase"):
            return f"({a[0]}).toLowerCase()"
        if n in ("substr", "substring"):
            if len(a) == 2:
                return f"({a[0]}).substring(({a[1]}) - 1)"
            return f"({a[0]}).substring(({a[1]}) - 1, ({a[1]}) - 1 + ({a[2]}))"
        if n == "concat":
            return "(" + " + ".join(f"String({x})" for x in a) + ")"
        if n in ("length", "char_length"):
            return f"({a[0]}).length"
        if n == "trim":
            return f"({a[0]}).trim()"
        if n == "abs":
            return f"Math.abs({a[0]})"
        if n in ("greatest", "least"):
            return f"Math.{'max' if n == 'greatest' else 'min'}({', '.join(a)})"
        if n in ("sqrt", "exp", "floor", "ceil", "sin", "cos", "tan", "log"):
            return f"Math.{n}({a[0]})"
        if n == "ceiling":
            return f"Math.ceil({a[0]})"
        if n in ("pow", "power"):
            return f"Math.pow({a[0]}, {a[1]})"
        if n == "pmod":
            return f"Math.pmod({a[0]}, {a[1]})"
        if n == "ln":
            return f"Math.log({a[0]})"
        if n == "round":
            return f"Math.round({a[0]})"
        if n == "coalesce":
            out = a[-1]
            for x in reversed(a[:-1]):
                out = f"(({x}) != null ? ({x}) : ({out}))"
            return out
        if n == "if":
            return f"(({a[0]}) ? ({a[1]}) : ({a[2]}))"
        if n in ("year", "month", "dayofmonth", "day", "hour", "minute", "second"):
            acc = {"year": "getYear", "month": "getMonthOfYear", "dayofmonth": "getDayOfMonth",
                   "day": "getDayOfMonth", "hour": "getHourOfDay", "minute": "getMinuteOfHour",
                   "second": "getSecondOfMinute"}[n]
            return f"org.joda.time.DateTime.parse({a[0]}).{acc}()"
        raise JSGenError(f"no JavaScript rendering for {n}()")
    raise JSGenError(f"no JavaScript rendering for {type(e).__name__}")


def js_function(params: List[str], body_expr: str) -> str:
    return f"function({', '.join(params)}) {{ return {body_expr}; }}"


def js_single_column_fn(e: A.Expr, ref: A.Ref, param: str) -> str:
    """``function(<dim>) {...}`` for a filter/extraction over one column (best effort text)."""
    try:
        body = js_expr(e, {ref.rid: param})
    except JSGenError:
        body = f"null /* evaluated natively over the dictionary: {e.sql()} */"
    return js_function([param], body)


def js_aggregator(kind: str, e: A.Expr, names: Dict[int, str], params: List[str]):
    """(fnAggregate, fnCombine, fnReset) for SUM/MIN/MAX over an arithmetic metric expression."""
    body = js_expr(e, names)
    if kind == "sum":
        agg = js_function(["current"] + params, f"current + ({body})")
        comb = "function(partialA, partialB) { return partialA + partialB; }"
        reset = "function() { return 0; }"
    elif kind in ("min", "max"):
        f = "Math.min" if kind == "min" else "Math.max"
        agg = js_function(["current"] + params, f"{f}(current, ({body}))")
        comb = f"function(partialA, partialB) {{ return {f}(partialA, partialB); }}"
        reset = ("function() { return Number.POSITIVE_INFINITY; }" if kind == "min"
                 else "function() { return Number.NEGATIVE_INFINITY; }")
    else:
        raise JSGenError(kind)
    return agg, comb, reset


def vm_compatible(e: A.Expr) -> bool:
    """Can the scan kernel's expression VM evaluate this metric expression?"""
    for x in e.walk():
        if isinstance(x, A.Ref):
            continue
        if isinstance(x, A.Lit):
            if not isinstance(x.value, (int, float)) or isinstance(x.value, bool):
                return False
            continue
        if isinstance(x, A.BinOp) and x.op in ("+", "-", "*", "/", "%"):
            continue
        if isinstance(x, A.UnOp) and x.op == "-":
            continue
        if isinstance(x, A.Cast) and (x.to in ("double", "float", "bigint", "int") or x.to.startswith("decimal")):
            if x.to in ("bigint", "int") and typeof(x.child) not in ("bigint", "int", "smallint", "tinyint"):
                return False
            continue
        if isinstance(x, A.Call) and x.name in ("abs", "greatest", "least", "floor", "ceil", "ceiling", "sqrt",
                                                  "log", "ln", "exp", "pow", "power", "pmod") and not x.is_agg:
            if x.name == "log" and len(x.args) != 1:
                return False
            continue
        return False
    return True
