"""Operator library: importing this package registers every op kernel."""
from . import io_ops, math_ops, nn_ops, optimizer_ops, sequence_ops, tensor_ops  # noqa: F401
from . import detection_ops, dist_ops, metric_ops, rnn_ops, structured_ops  # noqa: F401
from . import control_flow_grad  # noqa: F401,E402  (grad makers for while / tensor arrays)
from . import concurrency_ops  # noqa: F401,E402  (CSP channels / go / select)
from . import compat_ops  # noqa: F401,E402  (recurrent / parallel_do / readers / nccl ops / fused variants)
