"""Module SPI: pluggable functions, logical rules, statement parsers and plan rules.

Parity: ``SparklineDataModule`` / ``ModuleLoader`` (``asql/sparklinedata/SparklineDataModule.scala:32-151``):
a module contributes ``registerFunctions``, ``logicalRules``, a command ``parser``, a
``parsedTransform`` and ``physicalRules``; extra modules are loaded by name from
``spark.sparklinedata.modules``.  Here a module is any Python object (usually a module) with some of:

  register_functions(session)           -> None  (use session.register_udf)
  logical_rules: [fn(plan, session) -> plan | None]   applied after the built-in optimizer
  parse(text, session) -> DataFrame | None            tried before the SQL grammar (commands)
  physical_rules: [fn(plan, session) -> plan | None]  applied after the Druid rewrite

Names in the conf are ``package.module`` or ``package.module:attribute``, comma separated.
"""
from __future__ import annotations

import importlib
from typing import Any, List


class BaseModule:
    """The built-in module (the reference's BaseModule): date/time functions and the Druid
    planner are always installed; this class documents the hook names."""

    name = "base"
    logical_rules: List[Any] = []
    physical_rules: List[Any] = []

    def register_functions(self, session) -> None:
        pass

    def parse(self, text, session):
        return None


def load_module(spec: str):
    spec = spec.strip()
    if ":" in spec:
        mod, attr = spec.split(":", 1)
        obj = getattr(importlib.import_module(mod), attr)
        return obj() if isinstance(obj, type) else obj
    return importlib.import_module(spec)


def load_modules(session) -> List[Any]:
    names = session.conf.get("spark.sparklinedata.modules") or ""
    mods = [BaseModule()]
    for n in [x for x in names.split(",") if x.strip()]:
        m = load_module(n)
        if hasattr(m, "register_functions"):
            m.register_functions(session)
        mods.append(m)
    return mods
