"""Parameter-server runtime: native TCP RPC (csrc/runtime/rpc.cc) + client/server wrappers."""
from .rpc import RPCClient, RPCServer, bytes_to_var, var_to_bytes  # noqa: F401
