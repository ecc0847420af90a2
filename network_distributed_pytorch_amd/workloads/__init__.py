"""Reference-compatible experiment entry points (one sub-package per reference directory).

=================================  ===========================================================
``ddp_guide``                      process-group init (+ toy-MLP dense step), file:// rendezvous
``ddp_guide_cifar10``              dense DP, ResNet (ref: ResNet-50), CIFAR-10-shape, batch 256
``ddp_powersgd_guide_cifar10``     PowerSGD DP, ResNet (ref: ResNet-152), rank 4, batch 512
``ddp_powersgd_distillBERT_IMDb``  PowerSGD DP, DistilBERT, IMDb-shape, rank 16, batch 16·N
=================================  ===========================================================

Each has ``ddp_init`` (module-level ``config`` dict + ``setup``/``run_task``/``cleanup``) and
``run_script`` (``-rank -cuda [-world_size -init_method]``), plus ``reducer`` /
``tensor_buffer`` / ``partition_helper`` re-exports where the reference directory has them.
"""
