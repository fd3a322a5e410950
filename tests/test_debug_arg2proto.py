"""Native debug strings (reference learn/base/debug.h) and the dmlc::Config
front end (learn/base/arg2proto.h)."""
import torch

from wormhole_amd import config
from wormhole_amd.config.schema import DifactoConfig, LinearConfig
from wormhole_amd.utils.debug import debug_str, debug_str_block


def test_debug_str_short_and_long():
    assert debug_str(torch.tensor([1, 2, 3])) == "[3]: 1 2 3 "
    s = debug_str(torch.arange(20))
    assert s == "[20]: 0 1 2 3 4 ... 15 16 17 18 19 "
    assert debug_str(torch.arange(20), m=2) == "[20]: 0 1 ... 18 19 "
    assert debug_str(torch.tensor([0.5, 1.5])) == "[2]: 0.5 1.5 "


def test_debug_str_block():
    keys = torch.tensor([3, 7, 9], dtype=torch.int64)
    off = torch.tensor([0, 2, 3], dtype=torch.int64)
    lab = torch.tensor([1.0, 0.0])
    s = debug_str_block(keys, off, None, lab)
    assert s == "label: [2]: 1 0 \noffset: [3]: 0 2 3 \nindex: [3]: 3 7 9 "
    s = debug_str_block(keys, off, torch.tensor([0.5, 1.0, 2.0]), lab)
    assert s.endswith("\nvalue: [3]: 0.5 1 2 ")


def test_arg2proto_roundtrip(tmp_path):
    text = """# dmlc config style
train_data = "data/train part"   # quoted, with a space
val_data = data/val
minibatch = 1000
lr_eta = 0.05
algo = FTRL
"""
    proto = config.arg2proto(text)
    assert proto.splitlines() == ['train_data: "data/train part"', "val_data: data/val",
                                  "minibatch: 1000", "lr_eta: 0.05", "algo: FTRL"]
    p = tmp_path / "a.conf"
    p.write_text(text.replace("val_data = data/val", 'val_data = "data/val"'))
    c = config.load_dmlc(LinearConfig, str(p))
    assert c.train_data == "data/train part" and c.minibatch == 1000
    assert abs(c.lr_eta - 0.05) < 1e-12


def test_arg2proto_nested_passthrough(tmp_path):
    text = 'train_data = "x"\nembedding {\n dim = 8\n threshold = 2\n}\n'
    p = tmp_path / "d.conf"
    p.write_text(text)
    c = config.load_dmlc(DifactoConfig, str(p))
    assert c.embedding[0].dim == 8 and c.embedding[0].threshold == 2
