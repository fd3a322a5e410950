"""Progress vectors and their printers, byte-compatible with the reference
tables (learn/linear/progress.h:8-36, learn/difacto/progress.h:8-42).

Progress is a list of doubles that workers report and the scheduler
sum-merges (reference ps::Root/Slave, learn/solver/iter_solver.h:62,92,132).
AUC/accuracy are means of per-minibatch values (reference convention).
"""


class LinearProgress:
    SIZE = 6  # objv, acc, auc, count, new_ex, new_w

    def __init__(self):
        self.ttl_ex = 0.0
        self.nnz_w = 0.0

    @staticmethod
    def head():
        return "  ttl #ex   inc #ex    |w|_0       logloss  accuracy     AUC"

    def line(self, d):
        objv, acc, auc, count, new_ex, new_w = d[:6]
        self.ttl_ex += new_ex
        self.nnz_w += new_w
        if new_ex == 0:
            return ""
        return "%8.3g  %8.3g  %11.6g  %8.6f  %8.6f  %8.6f" % (
            self.ttl_ex, new_ex, self.nnz_w, objv / new_ex, acc / count, auc / count)

    @staticmethod
    def objv_per_ex(d):
        return d[0] / d[4] if d[4] else 0.0


class DifactoProgress:
    SIZE = 8  # objv, auc, objv_w, copc, count, new_ex, new_w, new_V

    def __init__(self):
        self.ttl_ex = 0.0
        self.nnz_w = 0.0
        self.nnz_V = 0.0  # reference leaves this uninitialised

    @staticmethod
    def head():
        return "  ttl #ex   inc #ex |  |w|_0  logloss_w |   |V|_0    logloss    AUC"

    def line(self, d):
        objv, auc, objv_w, copc, count, new_ex, new_w, new_V = d[:8]
        self.ttl_ex += new_ex
        self.nnz_w += new_w
        self.nnz_V += new_V
        if new_ex == 0:
            return ""
        return "%9.4g  %7.2g | %9.4g  %6.4f | %9.4g  %7.5f  %7.5f " % (
            self.ttl_ex, new_ex, self.nnz_w, objv_w / new_ex, self.nnz_V, objv / new_ex,
            auc / count)

    @staticmethod
    def objv_per_ex(d):
        return d[0] / d[5] if d[5] else 0.0


def merge(a, b):
    if a is None:
        return list(b)
    return [x + y for x, y in zip(a, b)]
