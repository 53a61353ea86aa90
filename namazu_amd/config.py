"""Config with viper-like semantics (reference: nmz/util/config/config.go).

Keys are case-insensitive and dotted ("explorePolicyParam.maxInterval").
Durations follow Go's time.ParseDuration (Go 1.10 src/time/format.go) through
spf13/cast.ToDuration: integers/floats are nanoseconds, strings without a unit
letter get "ns" appended.
"""
import copy
import datetime

try:
    import tomllib as _toml
except ImportError:  # Python 3.10
    import tomli as _toml

_UNITS = {
    "ns": 1, "us": 1000, "µs": 1000, "μs": 1000, "ms": 1000_000,
    "s": 1000_000_000, "m": 60 * 1000_000_000, "h": 3600 * 1000_000_000,
}
_I64MAX = (1 << 63) - 1


class DurationError(ValueError):
    pass


def parse_duration(s: str) -> int:
    """Go time.ParseDuration (Go 1.10): returns int nanoseconds."""
    orig = s
    neg = False
    if s and s[0] in "+-":
        neg = s[0] == "-"
        s = s[1:]
    if s == "0":
        return 0
    if s == "":
        raise DurationError("time: invalid duration " + orig)
    d = 0
    while s:
        if not (s[0] == "." or s[0].isdigit()):
            raise DurationError("time: invalid duration " + orig)
        # leadingInt
        i = 0
        v = 0
        while i < len(s) and s[i].isdigit():
            if v > _I64MAX // 10:
                raise DurationError("time: invalid duration " + orig)
            v = v * 10 + int(s[i])
            if v > _I64MAX:
                raise DurationError("time: invalid duration " + orig)
            i += 1
        pre = i > 0
        s = s[i:]
        post = False
        f, scale = 0, 1.0
        if s and s[0] == ".":
            s = s[1:]
            i = 0
            overflow = False
            while i < len(s) and s[i].isdigit():
                if not overflow:
                    if f > _I64MAX // 10:
                        overflow = True
                    else:
                        y = f * 10 + int(s[i])
                        if y > _I64MAX:
                            overflow = True
                        else:
                            f = y
                            scale *= 10
                i += 1
            post = i > 0
            s = s[i:]
        if not pre and not post:
            raise DurationError("time: invalid duration " + orig)
        i = 0
        while i < len(s) and not (s[i] == "." or s[i].isdigit()):
            i += 1
        if i == 0:
            raise DurationError("time: missing unit in duration " + orig)
        u, s = s[:i], s[i:]
        if u not in _UNITS:
            raise DurationError(f"time: unknown unit {u} in duration {orig}")
        unit = _UNITS[u]
        if v > _I64MAX // unit:
            raise DurationError("time: invalid duration " + orig)
        v *= unit
        if f > 0:
            v += int(float(f) * (float(unit) / scale))
            if v > _I64MAX:
                raise DurationError("time: invalid duration " + orig)
        d += v
        if d > _I64MAX:
            raise DurationError("time: invalid duration " + orig)
    return -d if neg else d


def to_duration(v) -> int:
    """spf13/cast.ToDuration."""
    if isinstance(v, bool):
        raise DurationError(f"unable to cast {v!r} to Duration")
    if isinstance(v, datetime.timedelta):
        return (v.days * 86400 + v.seconds) * 1000_000_000 + v.microseconds * 1000
    if isinstance(v, int):
        return v
    if isinstance(v, float):
        return int(v)
    if isinstance(v, str):
        if any(c in v for c in "nsuµmh"):
            return parse_duration(v)
        return parse_duration(v + "ns")
    raise DurationError(f"unable to cast {v!r} to Duration")


def _lower_keys(d):
    if isinstance(d, dict):
        return {str(k).lower(): _lower_keys(v) for k, v in d.items()}
    return d


class Config:
    """viper.Viper subset used by explore policies and storages."""

    DEFAULTS = {"explorepolicy": "random", "explorepolicyparam": {}}

    def __init__(self, data=None):
        self._m = copy.deepcopy(self.DEFAULTS)
        if data:
            for k, v in _lower_keys(data).items():
                self._m[k] = v

    @classmethod
    def from_toml(cls, text):
        return cls(_toml.loads(text))

    @classmethod
    def from_file(cls, path):
        with open(path, "rb") as f:
            return cls(_toml.load(f))

    def _find(self, key):
        node = self._m
        for part in key.lower().split("."):
            if not isinstance(node, dict) or part not in node:
                return False, None
            node = node[part]
        return True, node

    def set(self, key, value):
        parts = key.lower().split(".")
        node = self._m
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = _lower_keys(value) if isinstance(value, dict) else value

    def is_set(self, key):
        return self._find(key)[0]

    def get(self, key):
        return self._find(key)[1]

    def get_string(self, key):
        v = self.get(key)
        return "" if v is None else str(v)

    def get_duration(self, key):
        v = self.get(key)
        return 0 if v is None else to_duration(v)

    def get_float64(self, key):
        v = self.get(key)
        return 0.0 if v is None else float(v)

    def get_int(self, key):
        v = self.get(key)
        return 0 if v is None else int(v)

    def get_bool(self, key):
        v = self.get(key)
        return bool(v) if v is not None else False

    def get_string_slice(self, key):
        v = self.get(key)
        if v is None:
            return None
        if isinstance(v, str):
            return v.split()
        return [str(x) for x in v]

    def all_settings(self):
        return copy.deepcopy(self._m)
