"""World-N worker for tests/test_gpu_cli.py::test_sharded_compress_multirank_gloo (one process per rank,
all on cuda:0, gloo for the gather): sharded_compress of one file (rank 0 writes the container to
dst) and sharded_decompress of the single-GPU container (rank 0 writes the file to dst + ".dec")."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main(src: str, dst: str) -> None:
    import torch.distributed as dist

    import avrecode_amd as avr
    from avrecode_amd import shard

    dist.init_process_group("gloo")
    try:
        with avr.Context(0) as ctx:
            out = shard.sharded_compress(ctx, Path(src).read_bytes())
            if dist.get_rank() == 0:
                Path(dst).write_bytes(out)
            else:
                assert out is None
            # every rank decompresses its slice range of the single-GPU container (the same bytes)
            avrc = ctx.compress(Path(src).read_bytes(), avr.MODEL_PARALLEL)
            dec = shard.sharded_decompress(ctx, avrc)
            if dist.get_rank() == 0:
                Path(dst + ".dec").write_bytes(dec)
            else:
                assert dec is None
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
