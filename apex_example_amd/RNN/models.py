"""``apex.RNN`` model factories: LSTM / GRU / ReLU / Tanh over the
MIOpen-backed ``nn`` RNNs, plus the multiplicative LSTM, whose recurrence MIOpen does
not provide.  The mLSTM computes the input-side projections of every timestep as one
GEMM per layer ([T*B, in] x [in, 5H]) before the time loop, leaving two small GEMMs
and the gate pointwise work per step.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn


class _Stacked(nn.Module):
    def __init__(self, rnn, hidden_size, output_size, bidirectional):
        super().__init__()
        self.rnn = rnn
        width = hidden_size * (2 if bidirectional else 1)
        self.proj = nn.Linear(width, output_size) if output_size not in (None, width) else None

    def forward(self, x, hidden=None):
        out, h = self.rnn(x, hidden)
        if self.proj is not None:
            out = self.proj(out)
        return out, h


def _make(kind, input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0,
          bidirectional=False, output_size=None):
    kw = dict(num_layers=num_layers, bias=bias, batch_first=batch_first, dropout=dropout,
              bidirectional=bidirectional)
    if kind == "LSTM":
        rnn = nn.LSTM(input_size, hidden_size, **kw)
    elif kind == "GRU":
        rnn = nn.GRU(input_size, hidden_size, **kw)
    else:
        rnn = nn.RNN(input_size, hidden_size, nonlinearity=kind, **kw)
    return _Stacked(rnn, hidden_size, output_size, bidirectional)


def LSTM(input_size, hidden_size, num_layers, **kw):  # noqa: N802 (apex names)
    return _make("LSTM", input_size, hidden_size, num_layers, **kw)


def GRU(input_size, hidden_size, num_layers, **kw):  # noqa: N802
    return _make("GRU", input_size, hidden_size, num_layers, **kw)


def ReLU(input_size, hidden_size, num_layers, **kw):  # noqa: N802
    return _make("relu", input_size, hidden_size, num_layers, **kw)


def Tanh(input_size, hidden_size, num_layers, **kw):  # noqa: N802
    return _make("tanh", input_size, hidden_size, num_layers, **kw)


class mLSTMCell(nn.Module):  # noqa: N801
    """m = (W_mx x) * (W_mh h); gates = W_x x + W_h m (+ b)."""

    def __init__(self, input_size, hidden_size, bias=True):
        super().__init__()
        self.hidden_size = hidden_size
        self.w_ih = nn.Linear(input_size, 4 * hidden_size, bias=bias)
        self.w_hh = nn.Linear(hidden_size, 4 * hidden_size, bias=False)
        self.w_mih = nn.Linear(input_size, hidden_size, bias=False)
        self.w_mhh = nn.Linear(hidden_size, hidden_size, bias=False)

    def forward(self, x, state):
        return self.recur(self.w_ih(x), self.w_mih(x), state)

    def input_proj(self, x):
        """(W_x x + b, W_mx x) for a whole sequence [T, B, in] in one GEMM."""
        H = self.hidden_size
        w = torch.cat([self.w_ih.weight, self.w_mih.weight])
        b = None
        if self.w_ih.bias is not None:
            b = torch.cat([self.w_ih.bias, self.w_ih.bias.new_zeros(H)])
        xa = F.linear(x, w, b)
        return xa[..., :4 * H], xa[..., 4 * H:]

    def recur(self, xg, xm, state):
        """One step from the precomputed input projections xg = W_x x + b, xm = W_mx x."""
        h, c = state
        m = xm * self.w_mhh(h)
        i, f, g, o = (xg + self.w_hh(m)).chunk(4, -1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
        h = torch.sigmoid(o) * torch.tanh(c)
        return h, c


class _MLSTM(nn.Module):
    def __init__(self, input_size, hidden_size, num_layers, bias=True, batch_first=False,
                 dropout=0, bidirectional=False, output_size=None):
        super().__init__()
        if bidirectional:
            raise ValueError("mLSTM is unidirectional")
        self.batch_first = batch_first
        self.dropout = dropout
        self.cells = nn.ModuleList([mLSTMCell(input_size if i == 0 else hidden_size, hidden_size,
                                              bias) for i in range(num_layers)])
        self.proj = (nn.Linear(hidden_size, output_size)
                     if output_size not in (None, hidden_size) else None)

    def forward(self, x, hidden=None):
        if self.batch_first:
            x = x.transpose(0, 1)
        T, B, _ = x.shape
        H = self.cells[0].hidden_size
        states = hidden if hidden is not None else [
            (x.new_zeros(B, H), x.new_zeros(B, H)) for _ in self.cells]
        out = x
        new_states = []
        for li, cell in enumerate(self.cells):
            h, c = states[li]
            xg, xm = cell.input_proj(out)
            ys = []
            for t in range(T):
                h, c = cell.recur(xg[t], xm[t], (h, c))
                ys.append(h)
            out = torch.stack(ys)
            if self.dropout and li + 1 < len(self.cells):
                out = F.dropout(out, self.dropout, self.training)
            new_states.append((h, c))
        if self.proj is not None:
            out = self.proj(out)
        if self.batch_first:
            out = out.transpose(0, 1)
        return out, new_states


def mLSTM(input_size, hidden_size, num_layers, **kw):  # noqa: N802
    return _MLSTM(input_size, hidden_size, num_layers, **kw)
