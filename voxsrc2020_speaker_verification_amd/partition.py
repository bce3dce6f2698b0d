"""Data-parallel sharding of the extraction map.

The reference shards each data set's scp into N contiguous blocks with Kaldi's
utils/split_scp.pl (prepare_data.sh:31-37 -> split_scp.pl:211-244): shard k
gets floor(n/N) lines, the first n mod N shards one more, in order; the
per-GPU arks are then concatenated in shard order (eval_inference_model.sh:38-39).
"""

from __future__ import annotations


def shard_bounds(n, N):
    """[(begin, end)] line ranges of split_scp.pl's normal (non --utt2spk) mode."""
    if n == 0:
        raise ValueError("empty input scp file")
    per = n // N
    if per < 1:
        raise ValueError("You are splitting into too many pieces! [reduce $nj]")
    rem = n - per * N
    out, pos = [], 0
    for k in range(N):
        cnt = per + (1 if k < rem else 0)
        out.append((pos, pos + cnt))
        pos += cnt
    return out


def shard(items, rank, world):
    b, e = shard_bounds(len(items), world)[rank]
    return items[b:e]


def split_scp(in_path, out_paths):
    with open(in_path) as f:
        lines = f.readlines()
    for (b, e), p in zip(shard_bounds(len(lines), len(out_paths)), out_paths):
        with open(p, "w") as f:
            f.writelines(lines[b:e])
