"""World-N worker for tests/test_gpu_cli.py::test_sharded_compress_multirank_gloo and
tests/test_gpu_chained.py (one process per rank, all on cuda:0, gloo for the gather): the sharded
compress of one file (rank 0 writes the container to dst) and the sharded decompress of the
single-GPU container (rank 0 writes the file to dst + ".dec").  model "P" (default): the parallel
model, slice ranges; "C": the chained model, chain ranges."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main(src: str, dst: str, model: str = "P") -> None:
    import torch.distributed as dist

    import avrecode_amd as avr
    from avrecode_amd import shard

    dist.init_process_group("gloo")
    try:
        with avr.Context(0) as ctx:
            data = Path(src).read_bytes()
            if model == "C":
                out = shard.sharded_compress_chained(ctx, data)
            else:
                out = shard.sharded_compress(ctx, data)
            if dist.get_rank() == 0:
                Path(dst).write_bytes(out)
            else:
                assert out is None
            # every rank decompresses its range of the single-GPU container (the same bytes)
            if model == "C":
                dec = shard.sharded_decompress_chained(ctx, ctx.compress(data, avr.MODEL_CHAINED))
            else:
                dec = shard.sharded_decompress(ctx, ctx.compress(data, avr.MODEL_PARALLEL))
            if dist.get_rank() == 0:
                Path(dst + ".dec").write_bytes(dec)
            else:
                assert dec is None
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main(*sys.argv[1:4])
