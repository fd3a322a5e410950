"""Typed configuration schemas of the PS learners.

Field names, defaults and enums mirror the reference protobuf schemas
(learn/linear/config.proto:6-134, learn/difacto/config.proto:6-167) so every
reference ``.conf`` file parses unchanged.  Unknown keys are fatal, exactly as
protobuf TextFormat's CHECK is in the reference (learn/base/arg_parser.h:36-45).
"""
from dataclasses import dataclass, field, fields
from typing import List

LOSS = {"SQUARE": 1, "LOGIT": 2, "SQUARE_HINGE": 4}
ALGO = {"SGD": 1, "ADAGRAD": 2, "FTRL": 3}


@dataclass
class LinearConfig:
    train_data: str = ""
    val_data: str = ""
    data_format: str = "libsvm"
    model_out: str = ""
    model_in: str = ""
    predict_out: str = ""
    loss: int = 2
    lambda_l1: float = 1.0
    lambda_l2: float = 0.0
    algo: int = 3
    minibatch: int = 1000
    max_data_pass: int = 10
    lr_eta: float = 0.01
    save_iter: int = -1
    load_iter: int = -1
    local_data: bool = False
    num_parts_per_file: int = 10
    rand_shuffle: int = 10
    neg_sampling: float = 1.0
    prob_predict: bool = True
    dropout: float = 0.0
    print_sec: float = 1.0
    lr_beta: float = 1.0
    num_threads: int = 2
    max_concurrency: int = 2
    key_cache: bool = True
    msg_compression: bool = True
    fixed_bytes: int = 0
    _set: set = field(default_factory=set, repr=False)

    ENUMS = {"loss": LOSS, "algo": ALGO}

    def has(self, name):
        return name in self._set


@dataclass
class Embedding:
    dim: int = 0
    threshold: int = 0
    lambda_l2: float = 0.0
    lr_eta: float = 0.01
    lr_beta: float = 1.0
    init_scale: float = 0.01
    dropout: float = 0.0
    grad_clipping: float = 0.0
    grad_normalization: float = 0.0
    _set: set = field(default_factory=set, repr=False)

    ENUMS = {}

    def has(self, name):
        return name in self._set


@dataclass
class DifactoConfig:
    train_data: str = ""
    val_data: str = ""
    data_format: str = "libsvm"
    model_out: str = ""
    model_in: str = ""
    predict_out: str = ""
    lambda_l1: float = 1.0
    lambda_l2: float = 0.0
    lr_eta: float = 0.01
    embedding: List[Embedding] = field(default_factory=list)
    minibatch: int = 1000
    max_data_pass: int = 10
    early_stop: bool = False
    save_iter: int = -1
    load_iter: int = -1
    local_data: bool = False
    num_parts_per_file: int = 10
    rand_shuffle: int = 10
    neg_sampling: float = 1.0
    prob_predict: bool = True
    print_sec: float = 1.0
    lr_beta: float = 1.0
    l1_shrk: bool = True
    max_objv: float = 0.0
    min_objv_decr: float = 1e-5
    num_threads: int = 2
    max_concurrency: int = 2
    key_cache: bool = True
    msg_compression: bool = True
    fixed_bytes: int = 0
    _set: set = field(default_factory=set, repr=False)

    ENUMS = {}
    NESTED = {"embedding": Embedding}

    def has(self, name):
        return name in self._set


def public_fields(cls):
    return [f for f in fields(cls) if not f.name.startswith("_")]
