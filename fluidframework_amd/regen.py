"""Building the resubmitted op of Client.regeneratePendingOp (client.ts:917-960) from the engine's
MTR_DELTA_REGEN / MTR_DELTA_REGEN_X records (include/mtr_types.h).

resetPendingDeltaToOps (client.ts:708-800) re-expresses each member of the pending group, in tree
order, at its reconnection position:

* INSERT -> ``createInsertSegmentOp(pos, segment)`` (opBuilder.ts:86-88): the member's piece of the
  original text (or the marker), with the op's own ``seg.props`` when it has them (client.ts:763-767),
  else the segment's current properties (``TextSegment.toJSONObject`` / ``Marker.toJSONObject``);
* REMOVE -> ``createRemoveRangeOp(pos, pos + cachedLength)``;
* ANNOTATE -> ``createAnnotateRangeOp(pos, pos + cachedLength, op.props, op.combiningOp)``;

one op per member, a GROUP when there is not exactly one (``createGroupOp``, client.ts:959).
"""
from __future__ import annotations

from typing import Any, Callable

import numpy as np

from . import abi
from .jsjson import parse


def records(deltas: np.ndarray) -> dict[int, list[tuple[int, int, int, int, int]]]:
    """Pair a document's delta records -> {record index: [(type, pos, len, text offset, props ref)]}."""
    out: dict[int, list] = {}
    d = np.asarray(deltas)
    k = 0
    while k < len(d):
        kind = int(d["kind"][k])
        if abi.DELTA_REGEN <= kind < abi.DELTA_REGEN + 3:
            if k + 1 >= len(d) or int(d["kind"][k + 1]) != abi.DELTA_REGEN_X:
                raise ValueError("MTR_DELTA_REGEN without its MTR_DELTA_REGEN_X record")
            out.setdefault(int(d["op"][k]), []).append(
                (kind - abi.DELTA_REGEN, int(d["pos"][k]), int(d["len"][k]), int(d["pos"][k + 1]), int(d["len"][k + 1])))
            k += 2
        else:
            k += 1
    return out


def props_dict(pairs: list[tuple[int, int]], interner) -> dict:
    """[(key id, value id)] -> the property object (JS own-key order kept)."""
    keys = {v: k for k, v in interner.keys.items()}
    vals = {v: k for k, v in interner.vals.items()}
    vals.update({v: k for k, v in interner.never.items()})
    return {keys[k]: parse(vals[v]) for k, v in pairs}


def _utf16_slice(s: str, off: int, n: int) -> str:
    b = s.encode("utf-16-le", "surrogatepass")
    return b[2 * off:2 * (off + n)].decode("utf-16-le", "surrogatepass")


def _member(reset_op: dict, rec: tuple, props_of: Callable[[int], dict]) -> dict:
    t, pos, n, off, ref = rec
    if t != reset_op.get("type"):
        raise ValueError("regenerate record does not match the op")
    if t == 1:
        return {"pos1": pos, "pos2": pos + n, "type": 1}
    if t == 2:
        op = {"pos1": pos, "pos2": pos + n, "props": reset_op.get("props"), "type": 2}
        if reset_op.get("combiningOp") is not None:
            op["combiningOp"] = reset_op["combiningOp"]
        return op
    seg = reset_op["seg"]
    own = isinstance(seg, dict) and "props" in seg  # resetOp.seg.props !== undefined
    props: Any = seg["props"] if own else (props_of(ref) if ref >= 0 else None)
    if isinstance(seg, dict) and "marker" in seg:
        spec: Any = {"marker": seg["marker"]}
        if props is not None:
            spec["props"] = props
    else:
        text = _utf16_slice(seg if isinstance(seg, str) else seg["text"], off, n)
        spec = {"text": text, "props": props} if props is not None else text
    return {"pos1": pos, "seg": spec, "type": 0}


def regenerated_op(reset_op: dict, recs: dict, first: int, props_of: Callable[[int], dict]) -> dict:
    """The op regeneratePendingOp returns for `reset_op` whose records start at index `first`
    (DocLog.regenerate's return value); props_of(ref) -> the properties a REGEN_X record references."""
    members = reset_op["ops"] if reset_op.get("type") == 3 else [reset_op]
    ops = []
    for k, m in enumerate(members):
        ops.extend(_member(m, r, props_of) for r in recs.get(first + k, []))
    return ops[0] if len(ops) == 1 else {"ops": ops, "type": 3}
