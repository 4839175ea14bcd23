"""The ``horovod`` import namespace is a pure alias of mivod (same objects)."""


def test_aliases_are_the_mivod_objects():
    import horovod
    import horovod.keras as hk
    import horovod.tensorflow.keras as htk
    import horovod.torch as ht

    import mivod
    import mivod.keras
    import mivod.torch

    assert ht.DistributedOptimizer is mivod.torch.DistributedOptimizer
    assert ht.init is mivod.init and horovod.init is mivod.init
    assert ht.Compression is mivod.Compression
    assert hk.DistributedOptimizer is mivod.keras.DistributedOptimizer
    assert htk.DistributedOptimizer is mivod.keras.DistributedOptimizer
    for cb in ("BroadcastGlobalVariablesCallback", "MetricAverageCallback",
               "LearningRateWarmupCallback", "LearningRateScheduleCallback"):
        assert getattr(hk.callbacks, cb) is getattr(mivod.keras.callbacks, cb)
        assert getattr(htk.callbacks, cb) is getattr(mivod.keras.callbacks, cb)
    for fn in ("allreduce", "allgather", "broadcast", "allreduce_async", "synchronize", "poll",
               "broadcast_parameters", "broadcast_optimizer_state", "rank", "size",
               "local_rank", "local_size", "cross_rank", "cross_size", "shutdown"):
        assert getattr(ht, fn) is getattr(mivod.torch, fn), fn
