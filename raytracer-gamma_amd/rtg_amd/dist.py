"""Row-cyclic frame sharding across ranks.

Rows are grouped in blocks of B rows; block b goes to rank b % G.  Every rank
renders its blocks packed in order (rtg_render_device with shard=rank,
nShards=G) into a buffer padded to the largest shard, rank 0 gathers the G
buffers with ONE collective (RCCL gather over xGMI), and `assemble` restores row
order with a single permute: shard g's local block lb is global block lb*G+g.
The camera uses global rows, so the assembled frame is bit-identical to a
1-GPU render.
"""
from __future__ import annotations


def n_blocks(height: int, row_block: int) -> int:
    return (height + row_block - 1) // row_block


def padded_rows(height: int, row_block: int, n_shards: int) -> int:
    """Rows of the largest shard, rounded to whole blocks (gather buffer size)."""
    nb = n_blocks(height, row_block)
    return ((nb + n_shards - 1) // n_shards) * row_block


def assemble(gathered, height: int, row_block: int):
    """gathered: [G, padded_rows, W, 3] (torch tensor or numpy array) -> [H, W, 3]."""
    G, R, W, C = gathered.shape
    nbmax = R // row_block
    x = gathered.reshape(G, nbmax, row_block, W, C)
    if hasattr(x, "permute"):
        x = x.permute(1, 0, 2, 3, 4)
    else:
        x = x.transpose(1, 0, 2, 3, 4)
    return x.reshape(nbmax * G * row_block, W, C)[:height]
