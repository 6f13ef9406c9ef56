"""NMT seq2seq LSTM (``nmt/nmt.cc:31-84``, graph ``nmt/rnn.cu:298-330``).

src words -> src embedding -> L encoder LSTM layers; dst words -> dst embedding -> L decoder LSTM
layers whose initial (h, c) are the encoder layer's final state; top decoder output -> linear
over the vocabulary -> softmax, trained with sparse CCE against the dst words (the reference's
softmaxDP node).  The sequence is cut into ``chunk``-step LSTM ops like the reference
(``LSTM_PER_NODE_LENGTH = 10``, ``nmt/rnn.h:23``) so every chunk can be placed independently.
Defaults: batch 64/worker, 2 layers, seq 20, hidden 2048, embed 2048, vocab 20K (``nmt.cc:34-45``).
"""
from __future__ import annotations

from dataclasses import dataclass

from flexmi.core.types import DataType


@dataclass
class NMTConfig:
    layers: int = 2
    seq: int = 20
    hidden: int = 2048
    embed: int = 2048
    vocab: int = 20 * 1024
    chunk: int = 10

    @staticmethod
    def small():
        return NMTConfig(layers=2, seq=6, hidden=16, embed=16, vocab=50, chunk=3)


def _lstm_stack(m, x, cfg, states=None, tag="enc"):
    """x [B, T, E] -> top output [B, T, H]; returns (y, [(h, c) per layer])."""
    finals = []
    for layer in range(cfg.layers):
        T = x.dims[1]
        sizes = [min(cfg.chunk, T - s) for s in range(0, T, cfg.chunk)]
        pieces = m.split(x, sizes, 1, name=f"{tag}{layer}.split") if len(sizes) > 1 else [x]
        h = c = None
        if states is not None:
            h, c = states[layer]
        ys = []
        for j, piece in enumerate(pieces):
            y, h, c = m.lstm(piece, cfg.hidden, h, c, name=f"{tag}{layer}.lstm{j}")
            ys.append(y)
        x = m.concat(ys, 1, name=f"{tag}{layer}.concat") if len(ys) > 1 else ys[0]
        finals.append((h, c))
    return x, finals


def nmt(model, cfg: NMTConfig = None, batch=None):
    cfg = cfg or NMTConfig()
    b = batch or model.config.batchSize
    T = cfg.seq
    src = model.create_tensor([b * T, 1], DataType.DT_INT32, name="src")
    dst = model.create_tensor([b * T, 1], DataType.DT_INT32, name="dst")
    se = model.embedding(src, cfg.vocab, cfg.embed, name="src_embed")
    de = model.embedding(dst, cfg.vocab, cfg.embed, name="dst_embed")
    se = model.reshape(se, [b, T, cfg.embed], name="src_seq")
    de = model.reshape(de, [b, T, cfg.embed], name="dst_seq")
    _, enc_states = _lstm_stack(model, se, cfg, None, "enc")
    dec, _ = _lstm_stack(model, de, cfg, enc_states, "dec")
    logits = model.dense(dec, cfg.vocab, name="linear")
    logits = model.reshape(logits, [b * T, cfg.vocab], name="logits")
    out = model.softmax(logits, name="softmax")
    return {"src": src, "dst": dst}, out


def nmt_strategy(model, num_gpus, mode="reference"):
    """Per-chunk placement strategies for the NMT graph (``nmt/nmt.cc:269-309`` set_global_config).

    ``reference``: what the reference ships -- the source-side embedding on GPU 0 and the
    target-side one on GPU 1 (its ``embed[i]`` configs, i < seq / LSTM_PER_NODE_LENGTH -> 0 else 1),
    every LSTM chunk, the vocabulary projection and the softmax data parallel over all GPUs.
    ``pipeline``: chunk (operator) parallelism -- encoder and decoder chunks of layer l, step
    block j on GPU (l * nchunks + j) mod num_gpus, each chunk whole (no sample split), so
    consecutive chunks of a layer hand their (h, c) state to the next GPU; embeddings follow their
    first chunk, projection + softmax stay data parallel.
    Returns {op name: ParallelConfig}; the simulator can cost either (tools/soap_report.py)."""
    from flexmi.core.types import OperatorType
    from flexmi.parallel.layout import ParallelConfig
    n = num_gpus
    st = {}
    lstm = [op for op in model.layers if op.op_type == OperatorType.OP_LSTM]
    if mode == "reference":
        st["src_embed"] = ParallelConfig([1, 1], [0])
        st["dst_embed"] = ParallelConfig([1, 1], [min(1, n - 1)])
        for op in lstm:
            st[op.name] = ParallelConfig.data_parallel(op.out_ndims, n)
        return st
    if mode != "pipeline":
        raise ValueError(mode)
    chunks = {}
    for op in lstm:                       # names "<enc|dec><layer>.lstm<chunk>"
        tag, rest = op.name.split(".lstm")
        layer = int(tag[3:])
        chunks.setdefault(tag[:3], []).append((layer, int(rest), op))
    for side in ("enc", "dec"):
        items = sorted(chunks.get(side, []), key=lambda x: (x[0], x[1]))
        nch = 1 + max((j for _, j, _ in items), default=0)
        for layer, j, op in items:
            dev = (layer * nch + j + (nch if side == "dec" else 0)) % n
            st[op.name] = ParallelConfig([1] * op.out_ndims, [dev])
        first = next((op for layer, j, op in items if layer == 0 and j == 0), None)
        if first is not None:
            st["src_embed" if side == "enc" else "dst_embed"] = ParallelConfig([1, 1], list(st[first.name].device_ids))
    return st
