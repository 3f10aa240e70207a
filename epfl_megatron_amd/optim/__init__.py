"""Optimizer construction (reference ``megatron/optimizer/__init__.py``)."""
from .. import global_vars
from .grad_scaler import ConstantGradScaler, DynamicGradScaler
from .optimizer import MegatronOptimizer
from .scheduler import OptimizerParamScheduler


def get_param_groups(modules, no_weight_decay_cond=None, scale_lr_cond=None, lr_mult=1.0):
    """Weight decay off for ``.bias`` names and 1-D params; optional lr scaling.

    Group order: [wd, wd-scaled-lr, no-wd, no-wd-scaled-lr] (non-empty only)."""
    wd_plain, wd_scaled, nowd_plain, nowd_scaled = [], [], [], []
    for module in modules:
        for name, param in module.named_parameters():
            if not param.requires_grad:
                continue
            if no_weight_decay_cond is not None:
                no_wd = no_weight_decay_cond(name, param)
            else:
                no_wd = name.endswith(".bias") or len(param.shape) == 1
            scale_lr = scale_lr_cond(name, param) if scale_lr_cond is not None else False
            if not no_wd and not scale_lr:
                wd_plain.append(param)
            elif not no_wd and scale_lr:
                wd_scaled.append(param)
            elif no_wd and not scale_lr:
                nowd_plain.append(param)
            else:
                nowd_scaled.append(param)
    groups = []
    for params, wd_mult, lm in ((wd_plain, 1.0, 1.0), (wd_scaled, 1.0, lr_mult),
                                (nowd_plain, 0.0, 1.0), (nowd_scaled, 0.0, lr_mult)):
        if params:
            groups.append({"params": params, "wd_mult": wd_mult, "lr_mult": lm})
    return groups


def get_megatron_optimizer(model, no_weight_decay_cond=None, scale_lr_cond=None, lr_mult=1.0):
    """``model``: list of DDP-wrapped chunks (local DDP is required)."""
    args = global_vars.get_args()
    groups = get_param_groups(model, no_weight_decay_cond, scale_lr_cond, lr_mult)
    grad_scaler = None
    if args.fp16 or args.loss_scale:
        if args.loss_scale:
            grad_scaler = ConstantGradScaler(args.loss_scale)
        else:
            grad_scaler = DynamicGradScaler(initial_scale=args.initial_loss_scale,
                                            min_scale=args.min_loss_scale, growth_factor=2.0,
                                            backoff_factor=0.5,
                                            growth_interval=args.loss_scale_window,
                                            hysteresis=args.hysteresis)
    return MegatronOptimizer(model, groups, args.optimizer, args.lr, args.weight_decay,
                             adam_beta1=args.adam_beta1, adam_beta2=args.adam_beta2,
                             adam_eps=args.adam_eps, sgd_momentum=args.sgd_momentum,
                             clip_grad=args.clip_grad,
                             log_num_zeros_in_grad=args.log_num_zeros_in_grad,
                             grad_scaler=grad_scaler,
                             use_distributed_optimizer=args.use_distributed_optimizer)
