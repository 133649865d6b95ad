"""The C-ABI library loads and exports every symbol include/zbhip.h declares (no GPU needed)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from zeebe_amd import abi, native
from zeebe_amd.engine import ELEMENT_DTYPE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "zbhip.h")).read()
    return sorted(set(re.findall(r"\b(zbhip_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = native.load()
    out = subprocess.check_output(["nm", "-D", "--defined-only", native.LIB_PATH]).decode()
    exported = set(re.findall(r" T (zbhip_\w+)", out))
    declared = set(_declared())
    assert declared <= exported, declared - exported
    assert set(native.SYMBOLS) == declared
    assert b"gfx950" in L.zbhip_build_info()


def test_library_contains_gfx950_code_object():
    blob = open(native.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the embedded HIP fat binary targets gfx950 only
    # (code-object target triples; rocPRIM's host code names other architectures in its tables)
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_struct_sizes_match_header():
    # compile a tiny C program against the header and compare layouts
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "zbhip.h"
int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(zbhip_command), sizeof(zbhip_doc_entry),
 sizeof(zbhip_record), sizeof(zbhip_config), sizeof(zbhip_stats), offsetof(zbhip_record, ordinal),
 offsetof(zbhip_record, aux), sizeof(zbhip_element), sizeof(zbhip_xpart_cmd), offsetof(zbhip_record, partition),
 offsetof(zbhip_xpart_cmd, kind)); return 0;}
'''
    d = os.path.join(ROOT, "build")
    os.makedirs(d, exist_ok=True)
    src = os.path.join(d, "sizes.c")
    exe = os.path.join(d, "sizes")
    open(src, "w").write(prog)
    subprocess.check_call(["gcc", "-I" + os.path.join(ROOT, "include"), src, "-o", exe])
    got = [int(x) for x in subprocess.check_output([exe]).split()]
    assert got == [C.sizeof(abi.Command), C.sizeof(abi.DocEntry), C.sizeof(abi.Record), C.sizeof(abi.Config),
                   C.sizeof(abi.Stats), abi.Record.ordinal.offset, abi.Record.aux.offset, ELEMENT_DTYPE.itemsize,
                   C.sizeof(abi.XpartCmd), abi.Record.partition.offset, abi.XpartCmd.kind.offset]


def test_open_without_gpu_fails_loudly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    from zeebe_amd.engine import Partition
    with pytest.raises(native.ZbhipError) as e:
        Partition(max_instances=16, max_commands=16)
    assert "ENODEV" in str(e.value)


def test_java_adapter_binds_exported_symbols():
    # adapter/src/main/java/.../ZbHip.java (the Panama FFM binding; no JDK in this image): every
    # downcall names a function declared in include/zbhip.h and exported by libzbhip.so
    src = open(os.path.join(ROOT, "adapter", "src", "main", "java", "io", "camunda", "zeebe", "zbhip",
                            "ZbHip.java")).read()
    names = re.findall(r'fn\(\s*"(zbhip_[a-z_]+)"', src)
    assert len(names) >= 20
    header = open(os.path.join(ROOT, "include", "zbhip.h")).read()
    lib = native.load()
    for n in names:
        assert re.search(r"\b%s\(" % n, header), n
        assert hasattr(lib, n), n
    # the struct sizes the binding documents
    assert C.sizeof(abi.Command) == 16 and C.sizeof(abi.DocEntry) == 16
    assert C.sizeof(abi.Record) == 80 and C.sizeof(abi.XpartCmd) == 48


# ValueType of protocol/src/main/resources/protocol.xml:23-53 (transcribed): the Java adapter compares
# drained rows against ValueType.value(), so the header, the Python mirror and the oracle must use the
# protocol's numbers (a push row with JOB_BATCH = 1 would fall into the adapter's default branch)
PROTOCOL_VALUE_TYPES = {"JOB": 0, "PROCESS_INSTANCE": 5, "INCIDENT": 6, "MESSAGE": 10, "MESSAGE_SUBSCRIPTION": 11,
                        "PROCESS_MESSAGE_SUBSCRIPTION": 12, "JOB_BATCH": 14, "TIMER": 15,
                        "MESSAGE_START_EVENT_SUBSCRIPTION": 16, "VARIABLE": 17,
                        "PROCESS_INSTANCE_CREATION": 19, "PROCESS_EVENT": 24, "PROCESS_INSTANCE_BATCH": 34}


def test_value_types_equal_protocol_values():
    src = open(os.path.join(ROOT, "include", "zbhip.h")).read()
    header = {m.group(1): int(m.group(2)) for m in re.finditer(r"ZBHIP_VT_([A-Z_]+)\s*=\s*(\d+)", src)}
    assert header == PROTOCOL_VALUE_TYPES
    for name, value in PROTOCOL_VALUE_TYPES.items():
        assert getattr(abi, "VT_" + name) == value, name
    assert "#define ZBHIP_VT_" not in src
