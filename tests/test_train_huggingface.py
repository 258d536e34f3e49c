"""HuggingFaceTrainer: two CPU workers (gloo) each run a transformers.Trainer on their shard of a
data.Dataset, metrics flow to the session, the final model is checkpointed and restored by the
predictor. Mirrors reference python/ray/train/tests/test_huggingface_trainer.py (tiny model,
random-init, no downloads)."""
import numpy as np


def _init(train_dataset, eval_dataset, **config):
    import torch
    import transformers

    torch.manual_seed(0)
    cfg = transformers.GPT2Config(vocab_size=32, n_positions=16, n_embd=16, n_layer=1, n_head=2)
    model = transformers.GPT2LMHeadModel(cfg)

    def collate(rows):
        ids = torch.as_tensor(np.stack([r["input_ids"] for r in rows]), dtype=torch.long)
        return {"input_ids": ids, "labels": ids}

    args = transformers.TrainingArguments(output_dir=config["out"], per_device_train_batch_size=4,
                                          num_train_epochs=config.get("epochs", 2), logging_steps=2,
                                          learning_rate=5e-3, report_to=[], save_strategy="no",
                                          use_cpu=True, disable_tqdm=True, dataloader_num_workers=0)
    return transformers.Trainer(model=model, args=args, train_dataset=train_dataset, eval_dataset=eval_dataset,
                                data_collator=collate)


def test_huggingface_trainer_two_workers(ray_shared, tmp_path):
    import ray_memory_management_amd.data as data
    from ray_memory_management_amd.air.config import RunConfig, ScalingConfig
    from ray_memory_management_amd.train.huggingface import HuggingFacePredictor, HuggingFaceTrainer

    seq = np.tile(np.arange(8, dtype=np.int64), 2)  # a learnable repeating pattern
    train = data.from_items([{"input_ids": seq} for _ in range(32)], parallelism=2)
    ev = data.from_items([{"input_ids": seq} for _ in range(8)], parallelism=2)
    t = HuggingFaceTrainer(_init, trainer_init_config={"out": str(tmp_path / "hf"), "epochs": 6},
                           scaling_config=ScalingConfig(num_workers=2, use_gpu=False),
                           run_config=RunConfig(local_dir=str(tmp_path / "runs")),
                           datasets={"train": train, "evaluation": ev})
    res = t.fit()
    assert res.error is None, res.error
    assert res.metrics["train_loss"] < 3.3 and "eval_loss" in res.metrics  # ln(32) = 3.47 at init
    assert len(res.metrics_history) >= 2 and res.checkpoint is not None
    import transformers

    pred = HuggingFacePredictor.from_checkpoint(res.checkpoint, model_cls=transformers.GPT2LMHeadModel)
    logits = pred.predict(seq[None, :8])
    assert logits.shape == (1, 8, 32)
