"""Event model for the decision path (reference: nmz/signal).

Only what the batch/online decision path consumes is modelled:
  * ReplayHint()          signal/event.go:47-53
  * EntityID(), Deferred() signal/signal.go:113-119, event.go:33-39
  * DefaultAction() / DefaultFaultAction() class   event.go:61-71,
    event_packet.go:45-47, event_filesystem.go:58-60, action_fault_*.go
  * Equals()              signal/signal.go:174-186 (uuid ignored)

Event hash (build-defined): evhash = FNV1a64 of the canonical JSON
of the event map without "uuid", canonicalised the way Go's encoding/json
marshals a map[string]interface{} decoded from JSON: keys sorted, no
whitespace, numbers as float64 ('f' format, shortest round-trip, 'e' format
below 1e-6 / from 1e21), strings with Go's HTML-safe escaping. Two events are
Equal exactly when their evhash inputs are equal, so evhash equality is
Event.Equals modulo 64-bit collisions.
"""
import json
import math
import re
import uuid as _uuid

FNV_OFFSET = 0xCBF29CE484222325
FNV_PRIME = 0x100000001B3
_M64 = (1 << 64) - 1

FAULTABLE_CLASSES = {"PacketEvent": "PacketFaultAction", "FilesystemEvent": "FilesystemFaultAction"}
OUT_OF_SCOPE_CLASSES = {"ProcSetEvent"}  # random policy routes these to procPolicy (host side)


def fnv1a64(data: bytes, h: int = FNV_OFFSET) -> int:
    """Host-side FNV-1a 64 (used only to canonicalise event identities)."""
    for b in data:
        h = ((h ^ b) * FNV_PRIME) & _M64
    return h


def _go_float(f: float) -> str:
    """strconv.AppendFloat as used by encoding/json's floatEncoder (Go 1.8+)."""
    if math.isinf(f) or math.isnan(f):
        raise ValueError("json: unsupported value")
    if f == 0:
        return "-0" if math.copysign(1.0, f) < 0 else "0"
    a = abs(f)
    r = repr(f)  # shortest round-trip digits (same choice as strconv with prec -1)
    if a < 1e-6 or a >= 1e21:  # 'e' format, exponent without leading zeros
        mant, _, exp = r.partition("e")
        e = int(exp)
        return f"{mant}e{'-' if e < 0 else '+'}{abs(e)}"
    if "e" in r:  # expand Python's exponent form into Go's 'f' form
        mant, _, exp = r.partition("e")
        e = int(exp)
        neg = mant.startswith("-")
        ip, _, fp = mant.lstrip("-").partition(".")
        digits = ip + fp
        point = len(ip) + e
        if point >= len(digits):
            s = digits + "0" * (point - len(digits))
        elif point <= 0:
            s = "0." + "0" * (-point) + digits
        else:
            s = digits[:point] + "." + digits[point:]
        return ("-" if neg else "") + s
    return r[:-2] if r.endswith(".0") else r


_PLAIN = re.compile(r'[^"\\<>&\x00-\x1f\u2028\u2029]*\Z')


def _go_string(s: str) -> str:
    if _PLAIN.match(s):  # nothing to escape (the common case): Go writes the string as is
        return '"' + s + '"'
    out = ['"']
    for ch in s:
        c = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch in "<>&" or c in (0x2028, 0x2029):
            out.append("\\u%04x" % c)
        elif c < 0x20:
            out.append({"\n": "\\n", "\r": "\\r", "\t": "\\t"}.get(ch, "\\u%04x" % c))
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def go_json(v) -> str:
    """encoding/json Marshal of a value decoded into interface{}."""
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, (int, float)):
        return _go_float(float(v))
    if isinstance(v, str):
        return _go_string(v)
    if isinstance(v, dict):
        return "{" + ",".join(_go_string(str(k)) + ":" + go_json(v[k]) for k in sorted(v)) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(go_json(x) for x in v) + "]"
    raise TypeError(f"unsupported JSON value {v!r}")


class Action:
    """Map-based action (BasicAction). The map follows the reference's constructors: InitSignal's keys
    (signal.go:80-87) plus, for actions tied to an event (EventAcceptanceAction, PacketFaultAction,
    FilesystemFaultAction: action_accept_event.go:40, action_fault_packet.go:43,
    action_fault_filesystem.go:43), a top-level "event_uuid". NopAction keeps the event only as its
    cause (action_nop.go:30-39), not in the map."""

    def __init__(self, cls, entity, event=None, option=None, record_event_uuid=True):
        self.m = {"class": cls, "entity": entity, "type": "action",
                  "uuid": str(_uuid.uuid4()), "option": dict(option or {})}
        if event is not None and record_event_uuid:
            self.m["event_uuid"] = event.ID()
        self._event = event

    def Class(self):
        return self.m["class"]

    def Event(self):
        return self._event

    def EntityID(self):
        return self.m["entity"]

    def JSONMap(self):
        return self.m


class Event:
    """Map-based event (BasicEvent); construct from a JSON map or string."""

    def __init__(self, m):
        self.m = dict(m)

    @classmethod
    def from_json(cls, s):
        m = json.loads(s)
        if not isinstance(m.get("class"), str):
            raise ValueError(f"bad json {m!r}")
        return cls(m)

    @classmethod
    def packet(cls, entity, src, dst, option=None, replay_hint=None, deferred=True):
        """signal.NewPacketEvent (event_packet.go:26-43)."""
        opt = {"src_entity": src, "dst_entity": dst}
        opt.update(option or {})
        m = {"uuid": str(_uuid.uuid4()), "entity": entity, "type": "event",
             "class": "PacketEvent", "deferred": deferred, "option": opt}
        if replay_hint is not None:
            m["replay_hint"] = replay_hint
        return cls(m)

    def ID(self):
        return self.m.get("uuid", "")

    def EntityID(self):
        return self.m.get("entity", "")

    def Class(self):
        return self.m.get("class", "")

    def Deferred(self):
        d = self.m.get("deferred")
        return d if isinstance(d, bool) else False

    def ReplayHint(self):
        h = self.m.get("replay_hint")
        return h if isinstance(h, str) else ""

    def SetReplayHint(self, hint):
        self.m["replay_hint"] = hint

    def DefaultAction(self):
        if self.Deferred():
            return Action("EventAcceptanceAction", self.EntityID(), self)
        return Action("NopAction", self.EntityID(), self, record_event_uuid=False)

    def DefaultFaultAction(self):
        cls = FAULTABLE_CLASSES.get(self.Class())
        if cls is None or not self.Deferred():
            return None
        return Action(cls, self.EntityID(), self)

    def faultable(self):
        return self.Class() in FAULTABLE_CLASSES and self.Deferred()

    def canonical_json(self):
        return go_json({k: v for k, v in self.m.items() if k != "uuid"})

    def evhash(self):
        return fnv1a64(self.canonical_json().encode())

    def Equals(self, other):
        a = {k: v for k, v in self.m.items() if k != "uuid"}
        b = {k: v for k, v in other.m.items() if k != "uuid"}
        return a == b

    def JSONMap(self):
        return self.m
