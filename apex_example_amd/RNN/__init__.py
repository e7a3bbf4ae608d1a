"""apex.RNN counterparts (apex@f3a960f8 apex/RNN/; deprecated
upstream): ``LSTM, GRU, ReLU, Tanh, mLSTM(input_size, hidden_size, num_layers,
bias=True, batch_first=False, dropout=0, bidirectional=False, output_size=None)``.
LSTM / GRU / ReLU / Tanh run ``torch.nn.LSTM/GRU/RNN`` (MIOpen RNN kernels on
ROCm) with an optional output projection; mLSTM (multiplicative LSTM, Krause
et al. 2016) is a Python cell loop.  Input [T, B, F] (or [B, T, F] with
batch_first); returns (output, hidden)."""
from .models import GRU, LSTM, ReLU, Tanh, mLSTM  # noqa: F401
