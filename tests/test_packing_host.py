"""skyrl_amd.packing.pack on CPU: the reference's unpad_input layout (model_wrapper.py:272-289)."""

import torch

from skyrl_amd.packing import pack
from skyrl_amd.trainer import _positions


def test_pack_left_and_right_padding():
    seq = torch.arange(1, 13).view(2, 6)
    att = torch.tensor([[0, 0, 1, 1, 1, 0],   # left-padded prompt, right-padded response
                        [1, 1, 1, 1, 1, 1]])
    p = pack(seq, att)
    assert p.input_ids.tolist() == [[3, 4, 5, 7, 8, 9, 10, 11, 12]]
    assert p.position_ids.tolist() == [[0, 1, 2, 0, 1, 2, 3, 4, 5]]
    assert p.cu_seqlens.tolist() == [0, 3, 9] and p.cu_seqlens.dtype == torch.int32
    assert p.max_len == 6
    # packed index of every valid padded position; positions match the padded path's ids
    valid = att.reshape(-1).bool()
    assert p.packed_of[valid].tolist() == list(range(9))
    assert torch.equal(p.position_ids[0], _positions(att).reshape(-1)[valid])
