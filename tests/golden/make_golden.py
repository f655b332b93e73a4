#!/usr/bin/env python3
"""Regenerate the committed golden vectors under tests/golden/.

Run in the build container (needs /root/reference):  python tests/golden/make_golden.py

* arith_recoded.json / arith_cabac.json: seeded op scripts run through the reference's own
  arithmetic_code.h compiled as-is (oracle/_ref/ref_arith, built by `make -C oracle ref`).
* container.json: Recoded messages serialised by the Python protobuf runtime from a descriptor
  built by hand from recode.proto (proto2) -- pins the hand-written wire codecs.
* fixtures.json / fields.json: sizes / SHA-256 of the oracle's .avrc for the fixture files, every
  model mode (R, P on the u64 coder, P32; regression pins).

The files hold data only (inputs and expected outputs); no reference source is stored.
"""
import hashlib
import json
import os
import random
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
GOLD = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT / "tests"))

from _oracle import lps_table, oracle_cli  # noqa: E402


def recoded_scripts():
    scripts = []
    for seed, n, skew in [(1, 200, 0), (2, 3000, 0), (3, 3000, 1), (4, 20000, 2), (5, 1, 0), (6, 0, 0)]:
        rng = random.Random(seed)
        ops = []
        for _ in range(n):
            if skew == 2:
                # long runs of near-certain symbols force long deferred-digit (carry) chains
                pos, neg = rng.choice([(1, 95), (95, 1), (48, 48), (1, 1)])
            else:
                pos, neg = rng.randint(1, 0x60), rng.randint(1, 0x60)
            p1 = pos / (pos + neg)
            sym = int(rng.random() < (p1 if skew == 0 else (1 - p1 if skew == 1 else p1)))
            ops.append(("s", sym, pos, neg))
        ops.append(("f", 0, 0, 0))
        scripts.append({"seed": seed, "ops": ops})
    return scripts


def cabac_scripts():
    scripts = []
    # test/arithmetic_code.cpp:16-31 known-answer sequence for a past CABAC encoder bug
    states = [15, 17, 106, 28, 16, 0, 10, 26, 33, 22, 35, 58, 44, 0, 0, 1, 3, 5]
    bits = [1, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 0, 1, 1, 1, 1, 1, 1]
    ops = [("d", bits[0], states[0], 0), ("t", 0, 0, 0)]
    ops += [("d", bits[i], states[i], 0) for i in range(1, len(bits))]
    ops += [("d", 0, 0, 0)] * 16
    ops += [("t", 1, 0, 0)]
    scripts.append({"seed": "kat", "ops": ops})
    for seed, n in [(11, 100), (12, 5000), (13, 30000)]:
        rng = random.Random(seed)
        ops = []
        for _ in range(n):
            r = rng.random()
            if r < 0.15:
                ops.append(("b", rng.randint(0, 1), 0, 0))
            elif r < 0.17:
                ops.append(("t", 0, 0, 0))
            else:
                st = rng.randint(0, 127)
                mps = st & 1
                # draw the bin roughly from the state's own probability
                p_lps = 0.5 * (0.949 ** (st >> 1))
                ops.append(("d", mps ^ int(rng.random() < p_lps), st, 0))
        ops.append(("t", 1, 0, 0))
        scripts.append({"seed": seed, "ops": ops})
    return scripts


def run_ref(kind, ops):
    ref = ROOT / "oracle" / "_ref" / "ref_arith"
    lines = [kind]
    if kind == "cabac":
        lines.append(" ".join(str(v) for v in lps_table()))
    for op in ops:
        if op[0] == "s":
            lines.append(f"s {op[1]} {op[2]} {op[3]}")
        elif op[0] == "d":
            lines.append(f"d {op[1]} {op[2]}")
        elif op[0] in "bt":
            lines.append(f"{op[0]} {op[1]}")
        else:
            lines.append("f")
    out = subprocess.run([str(ref)], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    res = out.stdout.split()
    if kind == "recoded":
        assert res[1:] == ["decode", "ok"], res
    return res[0] if res and res[0] not in ("decode",) else ""


def container_golden():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "recode_golden.proto"
    fdp.syntax = "proto2"
    rec = fdp.message_type.add()
    rec.name = "Recoded"
    md = rec.nested_type.add()
    md.name = "Metadata"
    F = descriptor_pb2.FieldDescriptorProto
    for num, name, typ in [(1, "version", F.TYPE_BYTES), (2, "source_commit", F.TYPE_BYTES),
                           (3, "binary_sha256", F.TYPE_BYTES), (4, "binary_timestamp", F.TYPE_INT64)]:
        md.field.add(name=name, number=num, type=typ, label=F.LABEL_OPTIONAL)
    blk = rec.nested_type.add()
    blk.name = "Block"
    for num, name, typ in [(1, "size", F.TYPE_INT64), (2, "literal", F.TYPE_BYTES), (3, "skip_coded", F.TYPE_BOOL),
                           (4, "cabac", F.TYPE_BYTES), (5, "length_parity", F.TYPE_BOOL),
                           (6, "last_byte", F.TYPE_BYTES)]:
        blk.field.add(name=name, number=num, type=typ, label=F.LABEL_OPTIONAL)
    rec.field.add(name="metadata", number=1, type=F.TYPE_MESSAGE, label=F.LABEL_OPTIONAL,
                  type_name=".Recoded.Metadata")
    rec.field.add(name="block", number=2, type=F.TYPE_MESSAGE, label=F.LABEL_REPEATED,
                  type_name=".Recoded.Block")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    Recoded = message_factory.GetMessageClass(pool.FindMessageTypeByName("Recoded"))
    cases = []
    rng = random.Random(7)

    def case(blocks, version=None):
        m = Recoded()
        if version is not None:
            m.metadata.version = version.encode()
        for b in blocks:
            pb = m.block.add()
            if "size" in b:
                pb.size = b["size"]
            if "literal" in b:
                pb.literal = bytes.fromhex(b["literal"])
            if "skip_coded" in b:
                pb.skip_coded = b["skip_coded"]
            if "cabac" in b:
                pb.cabac = bytes.fromhex(b["cabac"])
            if "length_parity" in b:
                pb.length_parity = b["length_parity"]
            if "last_byte" in b:
                pb.last_byte = bytes.fromhex(b["last_byte"])
        cases.append({"blocks": blocks, "version": version, "bytes": m.SerializeToString().hex()})

    case([{"literal": ""}])
    case([{"size": 1000, "cabac": "1234", "length_parity": False, "last_byte": "80"}])
    case([{"size": 5, "skip_coded": True}])
    for _ in range(20):
        blocks = []
        for _ in range(rng.randint(1, 12)):
            t = rng.randint(0, 2)
            if t == 0:
                blocks.append({"literal": bytes(rng.randrange(256) for _ in range(rng.choice([0, 3, 200, 1500]))).hex()})
            elif t == 1:
                sz = rng.choice([8, 9, 300, 1 << 20, (1 << 35) + 3])
                blocks.append({"size": sz, "cabac": bytes(rng.randrange(256) for _ in range(rng.randint(0, 300))).hex(),
                               "length_parity": bool(sz & 1), "last_byte": "%02x" % rng.randrange(256)})
            else:
                blocks.append({"size": rng.randint(0, 1 << 40), "skip_coded": True})
        case(blocks, version=rng.choice([None, "avrecode-amd:P", "avrecode-amd:P64", "avrecode-amd:P32"]))
    return cases


def main():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "all", "ref"], check=True)
    rec = [{"seed": s["seed"], "ops": s["ops"], "expect": run_ref("recoded", s["ops"])} for s in recoded_scripts()]
    (GOLD / "arith_recoded.json").write_text(json.dumps(rec))
    cab = [{"seed": s["seed"], "ops": s["ops"], "expect": run_ref("cabac", s["ops"])} for s in cabac_scripts()]
    (GOLD / "arith_cabac.json").write_text(json.dumps(cab))
    (GOLD / "container.json").write_text(json.dumps(container_golden()))
    fx = []
    for name in ["realshort.mp4", "cockatoo.mp4"]:
        for mode in ["R", "P", "P32", "C"]:
            data = oracle_cli("compress", ROOT / "tests" / "fixtures" / name, mode=mode)
            fx.append({"file": name, "mode": mode, "avrc_len": len(data), "avrc_sha256": hashlib.sha256(data).hexdigest()})
    (GOLD / "fixtures.json").write_text(json.dumps(fx, indent=1))
    # fields.json: the field-coded fixtures' containers (the entries' descriptions are kept)
    fields = json.loads((GOLD / "fields.json").read_text())
    for e in fields["files"]:
        for mode in ["R", "P", "P32", "C"]:
            data = oracle_cli("compress", ROOT / "tests" / "fixtures" / e["file"], mode=mode)
            e[mode] = {"avrc_len": len(data), "avrc_sha256": hashlib.sha256(data).hexdigest()}
    (GOLD / "fields.json").write_text(json.dumps(fields, indent=1) + "\n")
    print("golden vectors written to", GOLD)


if __name__ == "__main__":
    main()
