"""Prometheus text-format parser (strict enough for tests, dashboards checks and the bench).

Validates what a Prometheus server would reject: every sample belongs to a family announced by
``# TYPE`` before it, families are contiguous, label values are properly escaped, no duplicate
series. Returns ``{family: {"type": t, "help": h, "samples": [(name, labels, value)]}}``.
"""

from __future__ import annotations

import math
import re
from typing import Dict, List, Tuple

_NAME = re.compile(r"[a-zA-Z_:][a-zA-Z0-9_:]*")


class PromParseError(ValueError):
    pass


def _parse_labels(s: str, pos: int) -> Tuple[Dict[str, str], int]:
    labels: Dict[str, str] = {}
    assert s[pos] == "{"
    pos += 1
    while True:
        if s[pos] == "}":
            return labels, pos + 1
        m = re.compile(r"[a-zA-Z_][a-zA-Z0-9_]*").match(s, pos)
        if not m:
            raise PromParseError(f"bad label name at {pos}: {s!r}")
        key = m.group(0)
        pos = m.end()
        if s[pos:pos + 2] != '="':
            raise PromParseError(f"expected =\" after {key}: {s!r}")
        pos += 2
        val = []
        while True:
            c = s[pos]
            if c == "\\":
                n = s[pos + 1]
                val.append({"\\": "\\", '"': '"', "n": "\n"}.get(n))
                if val[-1] is None:
                    raise PromParseError(f"bad escape \\{n}")
                pos += 2
            elif c == '"':
                pos += 1
                break
            elif c == "\n":
                raise PromParseError("newline in label value")
            else:
                val.append(c)
                pos += 1
        if key in labels:
            raise PromParseError(f"duplicate label {key}")
        labels[key] = "".join(val)
        if s[pos] == ",":
            pos += 1


def _base_family(name: str, families: Dict[str, dict]) -> str:
    if name in families:
        return name
    for suf in ("_bucket", "_sum", "_count", "_total", "_created"):
        if name.endswith(suf) and name[: -len(suf)] in families:
            return name[: -len(suf)]
    return name


def parse(text: str) -> Dict[str, dict]:
    families: Dict[str, dict] = {}
    order: List[str] = []
    seen_series = set()
    current = None
    for ln, line in enumerate(text.split("\n"), 1):
        if not line:
            continue
        if line.startswith("# HELP "):
            name, _, help_ = line[7:].partition(" ")
            families.setdefault(name, {"type": "untyped", "help": "", "samples": []})["help"] = help_
            continue
        if line.startswith("# TYPE "):
            name, _, typ = line[7:].partition(" ")
            if name in families and families[name]["samples"]:
                raise PromParseError(f"line {ln}: TYPE for {name} after its samples")
            if name in order:
                raise PromParseError(f"line {ln}: family {name} declared twice")
            families.setdefault(name, {"type": "untyped", "help": "", "samples": []})["type"] = typ
            order.append(name)
            current = name
            continue
        if line.startswith("#"):
            continue
        m = _NAME.match(line)
        if not m:
            raise PromParseError(f"line {ln}: bad metric name: {line!r}")
        name = m.group(0)
        pos = m.end()
        labels: Dict[str, str] = {}
        if pos < len(line) and line[pos] == "{":
            labels, pos = _parse_labels(line, pos)
        if pos >= len(line) or line[pos] != " ":
            raise PromParseError(f"line {ln}: expected space before value: {line!r}")
        parts = line[pos + 1:].split(" ")
        v = parts[0]
        value = {"+Inf": math.inf, "-Inf": -math.inf, "NaN": math.nan}.get(v)
        if value is None:
            value = float(v)
        fam = _base_family(name, families)
        if fam != current:
            raise PromParseError(f"line {ln}: sample {name} outside its family block (current {current})")
        key = (name, tuple(sorted(labels.items())))
        if key in seen_series:
            raise PromParseError(f"line {ln}: duplicate series {key}")
        seen_series.add(key)
        families[fam]["samples"].append((name, labels, value))
    return families


def values(families: Dict[str, dict], name: str, **match) -> List[float]:
    fam = families.get(_base_family(name, families), {"samples": []})
    out = []
    for n, labels, v in fam["samples"]:
        if n != name:
            continue
        if all(labels.get(k) == str(val) for k, val in match.items()):
            out.append(v)
    return out


def one(families: Dict[str, dict], name: str, **match) -> float:
    vs = values(families, name, **match)
    if len(vs) != 1:
        raise KeyError(f"{name} {match}: expected 1 sample, got {len(vs)}")
    return vs[0]
