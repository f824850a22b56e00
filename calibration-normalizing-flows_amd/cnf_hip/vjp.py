"""Reverse mode of the fused coupling stack (cnf_vjp in include/cnf.h)."""


def stack_vjp(stack, x, g_out, g_ld, all_grads, need_dx):
    raise NotImplementedError("native coupling VJP not built yet")
