"""JS-exact serialization edge cases of fluidframework_amd.jsjson (the host writer of every property
value and client id that lands in a summary blob).  Expected strings are what
ECMAScript's Number::toString / JSON.stringify / Object.keys produce (ES2019+): the reference writes
blobs with JSON.stringify (shared-object-base/src/serializer.ts:117)."""
import pytest

from fluidframework_amd.jsjson import array_index, js_key_order, js_number, js_string, js_stringify, parse

NUMBERS = [
    (0, "0"), (-0.0, "0"), (1, "1"), (-1, "-1"), (100, "100"), (1.0, "1"), (1.5, "1.5"), (-1.5, "-1.5"),
    (0.1, "0.1"), (0.1 + 0.2, "0.30000000000000004"), (1 / 3, "0.3333333333333333"), (4.35, "4.35"),
    (123456789, "123456789"), (2 ** 53 - 1, "9007199254740991"), (2 ** 53, "9007199254740992"),
    (2 ** 53 + 2, "9007199254740994"), (1e20, "100000000000000000000"),
    (123456789012345680000.0, "123456789012345680000"), (1e21, "1e+21"), (-1e21, "-1e+21"),
    (1.5e21, "1.5e+21"), (1e301, "1e+301"), (1.7976931348623157e308, "1.7976931348623157e+308"),
    (0.000001, "0.000001"), (1.2e-6, "0.0000012"), (5e-7, "5e-7"), (1e-7, "1e-7"), (-1.5e-10, "-1.5e-10"),
    (123e-20, "1.23e-18"), (5e-324, "5e-324"), (2.5e-5, "0.000025"),
    (float("nan"), "null"), (float("inf"), "null"), (float("-inf"), "null"),
]


@pytest.mark.parametrize("v,want", NUMBERS, ids=[w for _, w in NUMBERS])
def test_js_number(v, want):
    assert js_number(v) == want


def test_parse_gives_doubles():
    """JSON.parse makes every number a double: big integers round, 1.0 is 1, -0 prints 0."""
    assert js_stringify(parse("[1.0, 1e2, -0, 9007199254740993, 1E21, 0.00000050]")) == \
        "[1,100,0,9007199254740992,1e+21,5e-7]"


STRINGS = [
    ("plain", '"plain"'), ('q"b\\s/', '"q\\"b\\\\s/"'), ("\b\f\n\r\t", '"\\b\\f\\n\\r\\t"'),
    ("\x00\x01\x1f", '"\\u0000\\u0001\\u001f"'), ("\x7f", '"\x7f"'), ("  ", '"  "'),
    ("\ud800", '"\\ud800"'), ("\udc00", '"\\udc00"'), ("a\ud83dz", '"a\\ud83dz"'),
    ("😀", '"😀"'), ("\u2028\u2029", '"\u2028\u2029"'), ("\ude00\ud83d", '"\\ude00\\ud83d"'), ("é€", '"é€"'),
]


@pytest.mark.parametrize("s,want", STRINGS, ids=[repr(s) for s, _ in STRINGS])
def test_js_string(s, want):
    """ES2019 well-formed JSON.stringify: short escapes, other C0 controls as lowercase \\u00xx,
    U+007F and U+2028/2029 raw, a lone surrogate as \\udxxx, a surrogate pair raw."""
    assert js_string(s) == want


def test_key_order():
    """Object.keys: canonical array indices (< 2^32 - 1) ascending first, the rest in insertion order."""
    keys = ["b", "a", "10", "2", "-1", "01", "4294967294", "4294967295", "1.5", "0"]
    assert js_key_order(keys) == ["0", "2", "10", "4294967294", "b", "a", "-1", "01", "4294967295", "1.5"]
    assert array_index("4294967294") == 4294967294 and array_index("4294967295") is None
    assert array_index("00") is None and array_index("0") == 0
    obj = parse('{"b": 1, "10": {"z": 0, "1": [true, null]}, "a": "x", "2": 2.50}')
    assert js_stringify(obj) == '{"2":2.5,"10":{"1":[true,null],"z":0},"b":1,"a":"x"}'


def test_duplicate_keys_keep_first_position_last_value():
    """JSON.parse of a duplicate key: the first key's position, the last key's value."""
    assert js_stringify(parse('{"a": 1, "b": 2, "a": 3}')) == '{"a":3,"b":2}'
