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


def chunk_bounds(n_blocks_shard: int, chunks: int, row_block: int, last_frac: float = 0.0):
    """Row bounds of a shard split into `chunks` chunks of whole row blocks
    (bench.py's pipelined gather): equal chunks (last_frac 0), or a last
    chunk of about last_frac of the shard and the rest split equally, so the
    gather left after the last render is short.  Every chunk holds >= 1 block."""
    nb, K = n_blocks_shard, max(1, min(chunks, n_blocks_shard))
    if last_frac <= 0.0 or K == 1:
        return [row_block * ((nb * c) // K) for c in range(K + 1)]
    lastb = max(1, min(nb - (K - 1), round(nb * last_frac)))
    head = nb - lastb
    return [row_block * ((head * c) // (K - 1)) for c in range(K)] + [row_block * nb]


def default_chunks(world: int):
    """(chunks, last_frac) of bench.py's N > 1 step, from the one-GPU
    rehearsals of rank 0's part (tools/chunk_rehearsal.py,
    profiles/r03/chunks_c3_*.json, chunk_rehearsal.txt): every chunk is a
    launch that ends with a tail of long waves, so a 4- or 8-way shard renders
    best in three chunks and a 2-way one in four, the last one short (15 % of
    the shard) so little of the gather is left after the last render."""
    return (4, 0.15) if world <= 2 else (3, 0.15)
