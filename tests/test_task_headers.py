"""Static zeebe:taskHeaders -> the customHeaders of a job worker's jobs (BpmnJobBehavior.java:194-248,
365-399; TaskHeadersTransformer.java:24-58).  The reference writes the entries in the iteration order of
the java.util.HashMap HeaderEncoder collects them into.  The compiler (zeebe_amd/csrc/compiler.cpp
encode_task_headers: document order stably sorted by the final bucket) and the oracle (zb_oracle.cpp
JHashMap: the three maps restated put by put, resizes and the JDK 21 pre-sized copy included) must agree
byte for byte; known HashMap orders pin both: buckets ascending ((h ^ h >>> 16) & 15 for up to 12 keys),
colliding keys ("Aa" / "BB": String.hashCode 2112) in insertion order, 13+ keys in a 32-bucket table.
MessageStartEventTest-style pins of the reference (JobWorkerElementTest.shouldCreateJobWithCustomHeaders
:174-194) check the entries only; parity through the device path is in tests/test_gpu_task_headers.py."""
import ctypes as C
import random

import pytest

from oracle.oracle import Oracle
from zeebe_amd import bpmn, native
from zeebe_amd.engine import _Csr, msgpack_string_map


def compiled_headers(xml):
    L = native.load()
    xml = xml.encode()
    csr, err = C.c_void_p(), C.create_string_buffer(512)
    rc = L.zbhip_compile_bpmn(xml, len(xml), 2251799813685249, 1, C.byref(csr), err, 512)
    if rc != 0:
        return rc, err.value.decode()
    try:
        c = C.cast(csr, C.POINTER(_Csr)).contents
        if not c.header_begin:
            return 0, [b""] * c.n_elements
        hb = [c.header_begin[i] for i in range(c.n_elements + 1)]
        raw = C.string_at(c.header_bytes, hb[-1])
        return 0, [raw[hb[e]:hb[e + 1]] for e in range(c.n_elements)]
    finally:
        L.zbhip_free_csr(csr)


def oracle_headers(xml):
    o = Oracle()
    p = o.deploy(xml, 2251799813685249, 1)
    t = o.process_tables()[p]
    return t["headers"]


def process(headers, mi=False):
    b = bpmn.createExecutableProcess("p").startEvent("s").serviceTask("task", "t")
    for k, v in headers:
        b.zeebeTaskHeader(k, v)
    if mi:
        b.multiInstance("[1,2]")
    return b.endEvent("e").done()


def entries(xml):
    rc, hs = compiled_headers(xml)
    assert rc == 0, hs
    assert hs == oracle_headers(xml)
    got = [msgpack_string_map(h) for h in hs if h]
    return got[0] if got else ()


def test_known_hashmap_orders():
    assert entries(process([("a", "b"), ("c", "d")])) == (("a", "b"), ("c", "d"))
    # "z" (122: bucket 10) after "a" (97: bucket 1), whatever the document order
    assert entries(process([("z", "1"), ("a", "2")])) == (("a", "2"), ("z", "1"))
    # String.hashCode("Aa") == String.hashCode("BB") == 2112: one bucket, insertion (document) order
    assert entries(process([("BB", "1"), ("Aa", "2")])) == (("BB", "1"), ("Aa", "2"))
    assert entries(process([("Aa", "1"), ("BB", "2")])) == (("Aa", "1"), ("BB", "2"))
    # "q" (113: bucket 1 of 16, 17 of 32) and "a" (97: bucket 1 of both): 13 keys make the table 32 wide
    keys = ["q", "a"] + ["k%d" % i for i in range(11)]
    got = [k for k, _ in entries(process([(k, "v") for k in keys]))]
    assert got.index("a") < got.index("q")
    assert entries(process([("q", "1"), ("a", "2")])) == (("q", "1"), ("a", "2"))  # 16 wide: one bucket


def test_invalid_and_empty_headers():
    # TaskHeadersTransformer.isValidHeader: empty keys / values dropped; none left: NO_HEADERS
    assert entries(process([("", "x"), ("k", "")])) == ()
    assert entries(process([("k", "v"), ("", "x")])) == (("k", "v"),)
    rc, _ = compiled_headers(process([("k", "v"), ("k", "w")]))  # Collectors.toMap: duplicate key
    assert rc != 0


def test_encoding_forms():
    # fixstr / str8 / str16 lengths, non-ASCII keys (UTF-16 hashCode), a multi-instance task's headers
    long_v, longer_v = "x" * 40, "y" * 300
    got = entries(process([("long", long_v), ("longer", longer_v), ("küche", "ü"), ("\U0001F600", "smile")]))
    assert dict(got) == {"long": long_v, "longer": longer_v, "küche": "ü", "\U0001F600": "smile"}
    rc, hs = compiled_headers(process([("a", "b")], mi=True))
    assert rc == 0 and hs == oracle_headers(process([("a", "b")], mi=True))
    assert [msgpack_string_map(h) for h in hs if h] == [(("a", "b"),)]


@pytest.mark.parametrize("seed", range(40))
def test_random_header_sets_agree(seed):
    rnd = random.Random(seed)
    alphabet = "abAB01_-xyzé"
    n = rnd.choice([1, 2, 3, 5, 8, 12, 13, 20, 30])
    keys = set()
    while len(keys) < n:
        keys.add("".join(rnd.choice(alphabet) for _ in range(rnd.randint(1, 6))))
    hs = [(k, "v%d" % i) for i, k in enumerate(sorted(keys, key=lambda _: rnd.random()))]
    xml = process(hs)
    rc, c = compiled_headers(xml)
    if rc != 0:  # a bucket a HashMap would treeify: both refuse
        with pytest.raises(Exception):
            oracle_headers(xml)
        return
    assert c == oracle_headers(xml)
    assert dict(msgpack_string_map([h for h in c if h][0])) == dict(hs)
