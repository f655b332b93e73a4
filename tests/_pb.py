"""recode.proto (/root/reference/recode.proto:1-19) as a Python protobuf message class, built from a
hand-written FileDescriptorProto (proto2, the reference's field numbers and types; protoc is absent).
Test infrastructure: the independent wire codec the product's containers are checked against."""
from functools import lru_cache


@lru_cache(None)
def recoded_class():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="recode_check.proto", syntax="proto2")
    rec = fdp.message_type.add(name="Recoded")
    md = rec.nested_type.add(name="Metadata")
    for num, name, typ in [(1, "version", F.TYPE_BYTES), (2, "source_commit", F.TYPE_BYTES),
                           (3, "binary_sha256", F.TYPE_BYTES), (4, "binary_timestamp", F.TYPE_INT64)]:
        md.field.add(name=name, number=num, type=typ, label=F.LABEL_OPTIONAL)
    blk = rec.nested_type.add(name="Block")
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
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("Recoded"))


def parse(avrc: bytes):
    m = recoded_class()()
    m.ParseFromString(avrc)
    return m


def describe(m) -> dict:
    """The fields present, in avr_container_describe's JSON shape."""
    out = {"version": m.metadata.version.hex() if m.HasField("metadata") else None, "blocks": []}
    for b in m.block:
        d = {}
        for f in ("size", "literal", "skip_coded", "cabac", "length_parity", "last_byte"):
            if b.HasField(f):
                v = getattr(b, f)
                d[f] = v.hex() if isinstance(v, bytes) else v
        out["blocks"].append(d)
    return out


def check_container(avrc: bytes, original: bytes | None = None):
    """Parse with the protobuf runtime, re-serialise byte-identical, check the block grammar of
    compressor::run (recode.cpp:1115-1125, 1275-1297): literal, then (cabac | skip) + literal per
    coded slice ..., one block type each; literals + coded sizes re-assemble the file length."""
    m = parse(avrc)
    assert m.SerializeToString() == avrc, "protobuf runtime re-serialises differently"
    total = 0
    for b in m.block:
        kinds = [b.HasField("literal"), b.HasField("cabac"), b.HasField("skip_coded")]
        assert sum(kinds) == 1, b
        if b.HasField("literal"):
            total += len(b.literal)
        elif b.HasField("cabac"):
            assert b.HasField("size") and b.size >= 8
            assert b.HasField("length_parity") and b.length_parity == (b.size & 1)
            total += b.size
    if original is not None:
        assert total == len(original)
    return m
