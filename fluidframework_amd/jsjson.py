"""JavaScript-exact JSON for property values and ids.

Summary blobs are ``JSON.stringify(chunk)`` (packages/dds/shared-object-base/src/serializer.ts:117,
packages/dds/merge-tree/src/test/testSerializer.ts:28-31), so every property value that ends up in a
blob must be re-serialized with ECMAScript semantics:

* ``JSON.parse`` turns every number into an IEEE double; ``Number.prototype.toString`` prints the
  shortest round-trip digits in the ES2019 layout (no ``.0``, exponent only below 1e-6 / from 1e21).
* object key order is JS own-key order: canonical array-index keys ascending, then the remaining keys
  in insertion order.
* strings are written as in ES2019 well-formed ``JSON.stringify``: short escapes, other control
  characters as lowercase ``\\u00xx``, lone surrogates as ``\\udxxx``, everything else raw UTF-8.

This module is host-side plumbing used to intern values before they reach the engine.
"""
from __future__ import annotations

import json
import math
import re
from typing import Any

_INDEX_RE = re.compile(r"^(0|[1-9][0-9]*)$")
_MAX_SAFE = 2 ** 53


def array_index(key: str) -> int | None:
    """Return the integer if ``key`` is a canonical JS array index (ToUint32 round-trip, < 2^32-1)."""
    if _INDEX_RE.match(key):
        v = int(key)
        if v < 4294967295:
            return v
    return None


def js_key_order(keys):
    """Order keys of an object the way ``Object.keys`` would enumerate them."""
    idx = []
    rest = []
    for k in keys:
        v = array_index(k)
        if v is None:
            rest.append(k)
        else:
            idx.append((v, k))
    idx.sort()
    return [k for _, k in idx] + rest


def js_number(v: float | int) -> str:
    """ECMAScript Number::toString(10) as used by JSON.stringify (non-finite -> null)."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        if abs(v) < _MAX_SAFE:
            return str(v)
        v = float(v)
    if math.isnan(v) or math.isinf(v):
        return "null"
    if v == 0:
        return "0"
    sign = "-" if v < 0 else ""
    r = repr(abs(v))  # shortest round-trip digits
    if "e" in r or "E" in r:
        mant, exp = r.lower().split("e")
        exp = int(exp)
    else:
        mant, exp = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # position of the decimal point relative to the start of `digits`
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    n = len(ip) - lead_zeros + exp
    digits = digits.rstrip("0") or "0"
    k = len(digits)
    if k <= n <= 21:
        s = digits + "0" * (n - k)
    elif 0 < n <= 21:
        s = digits[:n] + "." + digits[n:]
    elif -6 < n <= 0:
        s = "0." + "0" * (-n) + digits
    else:
        e = n - 1
        es = ("+" if e >= 0 else "-") + str(abs(e))
        s = digits[0] + ("." + digits[1:] if k > 1 else "") + "e" + es
    return sign + s


_ESC = {
    '"': '\\"',
    "\\": "\\\\",
    "\b": "\\b",
    "\f": "\\f",
    "\n": "\\n",
    "\r": "\\r",
    "\t": "\\t",
}


def js_string(s: str) -> str:
    """JSON.stringify(string) as a Python str (lone surrogates escaped, pairs kept)."""
    out = ['"']
    i = 0
    n = len(s)
    while i < n:
        c = s[i]
        o = ord(c)
        if c in _ESC:
            out.append(_ESC[c])
        elif o < 0x20:
            out.append("\\u%04x" % o)
        elif 0xD800 <= o <= 0xDBFF:
            if i + 1 < n and 0xDC00 <= ord(s[i + 1]) <= 0xDFFF:
                out.append(c + s[i + 1])
                i += 1
            else:
                out.append("\\u%04x" % o)
        elif 0xDC00 <= o <= 0xDFFF:
            out.append("\\u%04x" % o)
        else:
            out.append(c)
        i += 1
    out.append('"')
    return "".join(out)


def to_utf8(s: str) -> bytes:
    """Encode a JS string (which may hold surrogate pairs as two code units) to UTF-8 bytes."""
    return s.encode("utf-16-le", "surrogatepass").decode("utf-16-le", "surrogatepass").encode(
        "utf-8", "surrogatepass"
    )


def js_stringify(v: Any) -> str:
    """JSON.stringify for a value produced by :func:`parse` (JS semantics)."""
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, (int, float)):
        return js_number(v)
    if isinstance(v, str):
        return js_string(v)
    if isinstance(v, list):
        return "[" + ",".join(js_stringify(x) for x in v) + "]"
    if isinstance(v, dict):
        return "{" + ",".join(js_string(k) + ":" + js_stringify(v[k]) for k in js_key_order(v.keys())) + "}"
    raise TypeError(f"unsupported JSON value {type(v)}")


def _norm_pairs(pairs):
    # JSON.parse keeps the last value of a duplicate key at the first key's position,
    # which is exactly dict() semantics.
    return dict(pairs)


def parse(text: str) -> Any:
    """JSON.parse with JS number semantics (every number is a double)."""
    return json.loads(
        text,
        object_pairs_hook=_norm_pairs,
        parse_int=lambda s: int(s) if abs(int(s)) < _MAX_SAFE else float(s),
        parse_float=float,
        parse_constant=lambda s: float(s),
    )


def plain_value(v: Any, nested: bool = False) -> bool:
    """True when matchProperties (properties.ts:71-105) is an equivalence on this value: no nested
    null and no empty object/array (a top-level null is a delete, not a value)."""
    if v is None:
        return not nested
    if isinstance(v, list):
        return len(v) > 0 and all(plain_value(x, True) for x in v)
    if isinstance(v, dict):
        return len(v) > 0 and all(plain_value(x, True) for x in v.values())
    return True


def eq_key(v: Any) -> str:
    """Canonical form used for matchProperties equivalence (properties.ts:71-105):
    deep equality that ignores object key order; numbers compared as doubles; an array compares
    like the object of its indices (matchProperties recurses with `for...in`)."""
    if isinstance(v, bool) or v is None:
        return json.dumps(v)
    if isinstance(v, (int, float)):
        f = float(v)
        if math.isnan(f):
            return "NaN#%d" % id(v)  # NaN never equals itself
        return "n" + repr(f if f != 0 else 0.0)
    if isinstance(v, str):
        return "s" + json.dumps(v)
    if isinstance(v, list):
        v = {str(i): x for i, x in enumerate(v)}
    if isinstance(v, dict):
        return "{" + ",".join(json.dumps(k) + ":" + eq_key(v[k]) for k in sorted(v.keys())) + "}"
    raise TypeError(f"unsupported JSON value {type(v)}")


def js_truthy(v: Any) -> bool:
    """ToBoolean of a JSON.parse value (None is JSON null)."""
    if v is None:
        return False
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float)):
        return v == v and v != 0
    if isinstance(v, str):
        return len(v) > 0
    return True


def utf16_less(a: str, b: str) -> bool:
    """a < b for two JS strings (code-unit order)."""
    return a.encode("utf-16-be", "surrogatepass") < b.encode("utf-16-be", "surrogatepass")
