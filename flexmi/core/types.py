"""Enumerations of the public API.

Integer values match the reference exactly so that strategy files, the C API and
user scripts written against FlexFlow keep working:
``include/ffconst.h:4-114`` (ActiMode .. OperatorType) and
``python/flexflow/core/flexflow_type.py:39-65`` (OpType codes of the torch ``.ff`` format).
"""
from enum import Enum, IntEnum

import torch


class ActiMode(IntEnum):
    AC_MODE_NONE = 10
    AC_MODE_RELU = 11
    AC_MODE_SIGMOID = 12
    AC_MODE_TANH = 13


class AggrMode(IntEnum):
    AGGR_MODE_NONE = 20
    AGGR_MODE_SUM = 21
    AGGR_MODE_AVG = 22


class PoolType(IntEnum):
    POOL_MAX = 30
    POOL_AVG = 31


class DataType(IntEnum):
    DT_FLOAT = 40
    DT_DOUBLE = 41
    DT_INT32 = 42
    DT_INT64 = 43
    DT_BOOLEAN = 44
    # MI355X extension: reduced-precision storage types (not in the reference).
    DT_BF16 = 45
    DT_HALF = 46


class LossType(IntEnum):
    LOSS_CATEGORICAL_CROSSENTROPY = 50
    LOSS_SPARSE_CATEGORICAL_CROSSENTROPY = 51
    LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE = 52
    LOSS_MEAN_SQUARED_ERROR_SUM_REDUCE = 53
    # extension: logistic loss used by MLPerf-style DLRM (sigmoid folded in)
    LOSS_BINARY_CROSSENTROPY = 54


class MetricsType(IntEnum):
    METRICS_ACCURACY = 1001
    METRICS_CATEGORICAL_CROSSENTROPY = 1002
    METRICS_SPARSE_CATEGORICAL_CROSSENTROPY = 1004
    METRICS_MEAN_SQUARED_ERROR = 1008
    METRICS_ROOT_MEAN_SQUARED_ERROR = 1016
    METRICS_MEAN_ABSOLUTE_ERROR = 1032


class OperatorType(IntEnum):
    """TASO-compatible operator codes (``include/ffconst.h:49-114``)."""
    OP_INPUT = 0
    OP_WEIGHT = 1
    OP_ANY = 2
    OP_CONV2D = 3
    OP_DROPOUT = 4
    OP_LINEAR = 5
    OP_BATCHMATMUL = 6
    OP_POOL2D = 7
    OP_RELU = 8
    OP_SIGMOID = 9
    OP_TANH = 10
    OP_ELU = 11
    OP_FLAT = 12
    OP_SOFTMAX = 13
    OP_BATCHNORM = 14
    OP_CONCAT = 15
    OP_SPLIT = 16
    OP_EMBEDDING = 17
    OP_RESHAPE = 18
    OP_REVERSE = 19
    OP_TRANSPOSE = 20
    OP_EW_ADD = 21
    OP_EW_MUL = 22
    OP_MATMUL = 23
    OP_MUL = 24
    OP_ENLARGE = 25
    OP_MERGE_GCONV = 26
    OP_CONSTANT_IMM = 27
    OP_CONSTANT_ICONV = 28
    OP_CONSTANT_ONE = 29
    OP_CONSTANT_POOL = 30
    OP_SQUEEZE = 31
    OP_UNSQUEEZE = 32
    OP_EW_SUB = 33
    OP_EW_DIV = 34
    OP_EW_EQUAL = 35
    OP_EW_GREATER = 36
    OP_EW_LESS = 37
    OP_EW_MAX = 38
    OP_EW_MIN = 39
    OP_REDUCE_ARGMAX = 40
    OP_REDUCE_ARGMIN = 41
    OP_REDUCE_MAX = 42
    OP_REDUCE_MEAN = 43
    OP_REDUCE_MIN = 44
    OP_REDUCE_PROD = 45
    OP_REDUCE_SUM = 46
    OP_PAD = 47
    OP_SHAPE = 48
    OP_SIZE = 49
    OP_TOPK = 50
    OP_WHERE = 51
    OP_CEIL = 52
    OP_CAST = 53
    OP_EXP = 54
    OP_ROUND = 55
    OP_LOG = 56
    OP_LOGICAL_NOT = 57
    OP_SQRT = 58
    OP_LEAKYRELU = 59
    OP_SLICE = 60
    OP_RESIZE = 61
    OP_PRELU = 62
    # flexmi extensions (values above the TASO range)
    OP_DOT_INTERACTION = 100
    OP_LSTM = 101
    OP_EMBEDDING_COLLECTION = 102
    OP_MSELOSS = 103


class OpType(IntEnum):
    """Op codes of the python frontends / torch ``.ff`` format
    (``python/flexflow/core/flexflow_type.py:39-65``)."""
    CONV2D = 2011
    EMBEDDING = 2012
    POOL2D = 2013
    LINEAR = 2014
    SOFTMAX = 2015
    CONCAT = 2016
    FLAT = 2017
    MSELOSS = 2020
    BATCH_NORM = 2021
    RELU = 2022
    SIGMOID = 2023
    TANH = 2024
    ELU = 2025
    DROPOUT = 2026
    BATCH_MATMUL = 2027
    SPLIT = 2028
    RESHAPE = 2029
    TRANSPOSE = 2030
    REVERSE = 2031
    EXP = 2040
    ADD = 2041
    SUBTRACT = 2042
    MULTIPLY = 2043
    DIVIDE = 2044
    INPUT = 2050
    OUTPUT = 2051
    # extensions
    DOT_INTERACTION = 2060
    LSTM = 2061


class ParameterSyncType(IntEnum):
    NONE = 80
    ALLREDUCE = 81  # RCCL all-reduce (the only mode on MI355X; PS mode of the reference is not used)


def enum_to_int(enum, item):
    """Reference helper (``flexflow_type.py:67-74``)."""
    return int(enum(item).value if not isinstance(item, Enum) else item.value)


def int_to_enum(enum, value):
    return enum(value)


_TORCH_DTYPES = {
    DataType.DT_FLOAT: torch.float32,
    DataType.DT_DOUBLE: torch.float64,
    DataType.DT_INT32: torch.int32,
    DataType.DT_INT64: torch.int64,
    DataType.DT_BOOLEAN: torch.bool,
    DataType.DT_BF16: torch.bfloat16,
    DataType.DT_HALF: torch.float16,
}


def to_torch_dtype(dt):
    return _TORCH_DTYPES[DataType(dt)]


def from_torch_dtype(td):
    for k, v in _TORCH_DTYPES.items():
        if v == td:
            return k
    raise KeyError(td)


def get_datatype_size(dt):
    return torch.tensor([], dtype=to_torch_dtype(dt)).element_size()
