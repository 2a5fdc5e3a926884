"""Drop-in for training/training.py: the Training driver, running every step
through the native executor (one fused forward+backward, one Adam launch)
instead of a TF1 Session.

Semantics kept from the reference:
  * loss = mean Keras categorical cross-entropy on the softmax outputs
    (:290-296), regularisation losses ignored (the reference's TODO);
  * tf.train.AdamOptimizer with the epsilon-hat update (:297-300);
  * streaming mean_loss / accuracy metrics, reset every epoch and before
    each evaluation (:316-354, :450-471);
  * per-layer gradient mean-norms ||g||_2 / size: for antisymmetric models
    conv1's kernel and each block's merged theta gradient (all its kernel
    variables, bias excluded; :385-409, generalised from the hard-coded
    20 variables per block); for regular models every rank>=4 kernel with
    spatial size >= 3 (:356-383);
  * CSV logs '{summaries_name}_{csv_logger_name}.csv' (global_step, metrics,
    gradient norms) every summaries_frequency steps and
    '{summaries_name}_evaluation_metrics.csv' after evaluations, space
    delimited, header written once (:186-217);
  * train(epochs, steps_per_epoch, learning_rate_schedule, ...) with the
    reference's arguments, evaluation and save policies (:473-668).

Data parallelism (one process per GPU, torch.distributed over RCCL): pass
rank/world-size-sharded datasets; parameters are broadcast from rank 0 at
construction, the flat fp32 gradient buffer is all-reduced (sum) once per
step and Adam applies it scaled by 1/world.  TensorBoard
summaries are not written (no TF); the CSV logs carry the same scalars.
"""
from __future__ import annotations

import csv
import json
import math
import os
import pathlib
import sys
import time

import numpy as np

from .. import distributed
from ..graph import Input, Model

__all__ = ["AdamOptimizer", "Training"]


class AdamOptimizer:
    """tf.train.AdamOptimizer(learning_rate, beta1, beta2, epsilon) — the
    hyper-parameters of the native asr_adam_update.  `learning_rate` is the
    default when train() gets no schedule."""

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, use_locking=False, name="Adam"):
        self.learning_rate = learning_rate
        self.beta1, self.beta2, self.epsilon = float(beta1), float(beta2), float(epsilon)
        self.name = name


def _dist():
    from .. import distributed
    if distributed.is_initialized():
        import torch.distributed as dist
        return dist
    return None


class Training:

    def __init__(self, model_build_function, kernel_type, optimizer, learning_rate_placeholder=None,
                 train_dataset=None, val_dataset=None, dataset_type="arrays", train_features_placeholder=None,
                 train_labels_placeholder=None, val_features_placeholder=None, val_labels_placeholder=None,
                 train_features=None, train_labels=None, val_features=None, val_labels=None, global_step=0,
                 num_layers=None, record_summaries=True, summaries=["mean_gradient_norms"], summaries_dir=None,
                 summaries_name=None, csv_logger_dir=None, csv_logger_name=None, dtype=None):
        import torch
        if train_dataset is None or not hasattr(train_dataset, "__iter__"):
            raise ValueError("train_dataset must be an ArrayDataset (dataset_utils) or another iterable of "
                             "(images, one-hot labels) device batches")
        if dataset_type not in ("tfrecords", "arrays"):
            raise ValueError("Supported values for argument `dataset_types` are 'tfrecords' (for TFRecordDatasets) "
                             "and 'arrays' (for datasets created from NumPy arrays).")
        self._torch = torch
        self.model_build_function = model_build_function
        self.kernel_type = kernel_type
        self.optimizer = optimizer if optimizer is not None else AdamOptimizer(epsilon=1e-7)
        self.learning_rate_placeholder = learning_rate_placeholder
        self.train_dataset = train_dataset
        self.val_dataset = val_dataset
        self.dataset_type = dataset_type
        self.num_layers = num_layers
        self.record_summaries = record_summaries
        self.summaries = summaries
        self.summaries_dir = summaries_dir
        self.summaries_name = summaries_name
        self.csv_logger_dir = csv_logger_dir
        self.csv_logger_name = csv_logger_name
        self.variables_updated = False
        self.eval_dataset = None
        self.training_loss = None
        self.best_training_loss = 99999999.9
        self.g_step = int(global_step)
        self.dist = _dist()
        self.world = self.dist.get_world_size() if self.dist else 1

        # model: the build function gets an Input of the dataset's batch shape
        img_shape, lbl_shape = self._batch_shapes(train_dataset)
        self.batch_size = img_shape[0]
        self.input_tensor = Input(shape=img_shape[1:], batch_size=img_shape[0])
        self.model = self.model_build_function(self.input_tensor)
        if not isinstance(self.model, Model):
            raise ValueError("The model_build_function you passed does not return a Model object.")
        self.native = self.model.compile_native(self.batch_size, dtype)
        if self.dist is not None:
            distributed.broadcast_params(self.native.params, 0)
            self.native.mark_updated()
        self._train_iter = iter(self.train_dataset)
        self._val_iter = iter(self.val_dataset) if self.val_dataset is not None else None
        dev = self.native.device
        self._accum = torch.zeros(4, dtype=torch.float32, device=dev)
        self._build_gradient_metrics()
        self._initialize_metrics()
        self.metric_values = [0.0, 0.0]
        if self.record_summaries:
            self._open_csv()

    # -- construction helpers --------------------------------------------------
    @staticmethod
    def _batch_shapes(ds):
        shapes = getattr(ds, "output_shapes", None)
        if shapes is None:
            raise ValueError("the dataset must expose output_shapes ((B,H,W,C), (B,K))")
        return tuple(shapes[0]), tuple(shapes[1])

    def _build_gradient_metrics(self):
        """Segments of the flat gradient buffer whose mean-norms are logged."""
        plan = self.native.plan
        off = 0
        segs, names = [], []
        layout = []
        for v in plan.weight_vars():
            layout.append((v, off))
            off += v.value.size
        pos = {id(v): o for v, o in layout}
        antisym = self.kernel_type == "antisymmetric"
        c1 = plan.conv1.kernel
        if antisym:
            segs.append((pos[id(c1)], pos[id(c1)] + c1.value.size))
            names.append(f"{plan.conv1.name}_kernel_gradient_mean_norm")
            blocks = plan.blocks if self.num_layers is None else plan.blocks[:self.num_layers]
            for conv in blocks:
                start = pos[id(conv.weights[0])]
                n = sum(w.value.size for w in conv.weights[:-1])  # theta, bias excluded
                segs.append((start, start + n))
                names.append(f"{conv.name}_kernel_gradient_mean_norm")
        else:
            for v, o in layout:
                if v.name.endswith("/kernel") and len(v.shape) >= 4 and v.shape[0] >= 3:
                    segs.append((o, o + v.value.size))
                    names.append(f"{v.name}_gradient_mean_norm")
        torch = self._torch
        offs = [s for s, _ in segs]
        ends = [e for _, e in segs]
        # contiguous segments [s_i, e_i): encode as consecutive offsets where
        # gaps are skipped by separate entries
        self._seg_bounds = torch.tensor(sorted(set(offs + ends)), dtype=torch.int64, device=self.native.device)
        bounds = self._seg_bounds.cpu().tolist()
        self._seg_index = [bounds.index(s) for s in offs]
        self._seg_sizes = [e - s for s, e in segs]
        self.gradient_mean_norm_names = names

    def _gradient_mean_norms(self, grads):
        from .. import runtime
        if not self.gradient_mean_norm_names:
            return []
        sq = runtime.segment_sq_norms(grads, self._seg_bounds).cpu().numpy().astype(np.float64)
        scale = 1.0 / self.world
        return [float(math.sqrt(sq[i]) * scale / n) for i, n in zip(self._seg_index, self._seg_sizes)]

    def _initialize_metrics(self):
        self.metric_names = ["mean_loss", "accuracy"]
        self.best_metric_values = [99999999.9, 0.0]

    def _open_csv(self):
        for what in ("summaries_dir", "summaries_name", "csv_logger_dir", "csv_logger_name"):
            if getattr(self, what) is None:
                raise ValueError(f"record_summaries=True needs `{what}`")
        pathlib.Path(self.csv_logger_dir).mkdir(parents=True, exist_ok=True)
        self._is_writer = (self.dist is None) or self.dist.get_rank() == 0

        def open_log(fname, header):
            if not self._is_writer:
                return None, None
            f = open(os.path.join(self.csv_logger_dir, fname), "a+", newline="")
            f.seek(0)
            empty = f.readline() == ""
            w = csv.writer(f, delimiter=" ")
            if empty:
                w.writerow(header)
                f.flush()
            return f, w

        self.csv_file_train, self.csv_writer_train = open_log(
            f"{self.summaries_name}_{self.csv_logger_name}.csv",
            ["global_step"] + self.metric_names + self.gradient_mean_norm_names)
        self.csv_file_val, self.csv_writer_val = open_log(f"{self.summaries_name}_evaluation_metrics.csv",
                                                          ["global_step"] + self.metric_names)

    # -- metrics ---------------------------------------------------------------
    def _reset_metrics(self):
        self._accum.zero_()

    def _metric_values(self):
        a = np.asarray(distributed.sum_over_ranks(self._accum.cpu().double().tolist()), dtype=np.float64)
        batches = max(a[3], 1.0)
        return [float(a[0] / batches), float(a[1] / max(a[2], 1.0))]

    # -- steps -------------------------------------------------------------------
    def _next(self, it_name):
        it = getattr(self, it_name)
        try:
            return next(it)
        except StopIteration:
            raise RuntimeError("dataset exhausted (use repeat=True for training)")

    def _targets(self, labels):
        """One-hot labels as the contiguous float32 device [N, K] tensor both
        the executor and the metrics kernel read (numpy, CPU or other-dtype
        batches are converted once here)."""
        torch = self._torch
        if isinstance(labels, np.ndarray):
            labels = torch.from_numpy(np.ascontiguousarray(labels))
        if not torch.is_tensor(labels):
            raise ValueError("labels must be a numpy array or a tensor of one-hot rows")
        t = labels.to(self.native.device, dtype=torch.float32, non_blocking=True).contiguous()
        if t.dim() != 2 or t.shape[0] != self.batch_size:
            raise ValueError(f"labels must be one-hot [{self.batch_size}, num_classes], got {tuple(t.shape)}")
        return t

    def train_step(self, learning_rate, with_norms=False):
        """One optimisation step on the next training batch; returns the
        gradient mean-norms when with_norms (else None)."""
        from .. import runtime
        images, labels = self._next("_train_iter")
        labels = self._targets(labels)
        loss, grads, probs = self.native.forward_backward(images, labels, want_probs=True)
        distributed.allreduce_grads(grads)
        norms = self._gradient_mean_norms(grads) if with_norms else None
        opt = self.optimizer
        self.native.apply_adam(grads, float(learning_rate), opt.beta1, opt.beta2, opt.epsilon,
                               grad_scale=1.0 / self.world)
        runtime.batch_metrics(probs, labels, loss, self._accum)
        self.g_step += 1
        self.variables_updated = True
        return norms

    def _check_device_status(self):
        """Once per epoch, after a synchronising read: launches completed, and
        the count of degraded in-launch slab hand-offs of the C=64 stacked
        backward (runtime.stack_status: a speed event, the gradients are
        exact) is kept in self.degraded_handoffs."""
        from .. import runtime
        if self.native is not None and hasattr(self.native, "check_status"):
            self.native.check_status()
        self.degraded_handoffs = getattr(self, "degraded_handoffs", 0) + runtime.stack_status(reset=True)

    def train(self, epochs, steps_per_epoch, learning_rate_schedule, eval_dataset="train", eval_frequency=5,
              eval_steps=None, save_during_training=False, save_dir=None, save_best_only=True, save_tags=["default"],
              save_name="", save_frequency=5, saver="train_saver", monitor="loss", summaries_frequency=10):
        from tqdm import trange
        if eval_dataset not in ("train", "val"):
            raise ValueError(f"`eval_dataset` must be one of 'train' or 'val', but is '{eval_dataset}'.")
        if eval_dataset == "val" and (self.val_dataset is None or eval_steps is None):
            raise ValueError("When eval_dataset == 'val', a `val_dataset` and `val_steps` must be passed.")
        self._initialize_metrics()
        if monitor == "loss":
            monitor = "mean_loss"
        if monitor not in self.metric_names:
            raise ValueError(f"You are trying to monitor {monitor}, which is not an available metric.")
        if eval_steps is None:
            eval_steps = steps_per_epoch
        self.eval_dataset = eval_dataset
        lr = learning_rate_schedule(self.g_step)
        show = (self.dist is None) or self.dist.get_rank() == 0
        for epoch in range(1, epochs + 1):
            tr = trange(steps_per_epoch, file=sys.stdout, disable=not show)
            tr.set_description(f"Epoch {epoch}/{epochs}")
            self._reset_metrics()
            for _ in tr:
                log = self.record_summaries and self.g_step % summaries_frequency == 0
                step_at = self.g_step
                norms = self.train_step(lr, with_norms=log)
                if log:
                    vals = self._metric_values()
                    if self.csv_writer_train is not None:
                        self.csv_writer_train.writerow([step_at] + vals + norms)
                        self.csv_file_train.flush()
                    tr.set_postfix(dict(zip(self.metric_names + ["global_step"], vals + [self.g_step])))
                lr = learning_rate_schedule(self.g_step)
            self.training_loss = self._metric_values()[0]  # (reads the device metrics: synchronises)
            self._check_device_status()
            evaluated = eval_frequency is not None and epoch % eval_frequency == 0
            if evaluated:
                desc = "Evaluation on training dataset" if eval_dataset == "train" else \
                    "Evaluation on validation dataset"
                self._evaluate(eval_dataset, eval_steps, desc)
                if self.record_summaries and self.csv_writer_val is not None:
                    self.csv_writer_val.writerow([self.g_step - 1] + self.metric_values)
                    self.csv_file_val.flush()
            if save_during_training and epoch % save_frequency == 0:
                save = True
                if save_best_only:
                    i = self.metric_names.index(monitor)
                    if monitor == "mean_loss":
                        save = self.metric_values[i] < self.best_metric_values[i]
                    else:
                        save = self.metric_values[i] > self.best_metric_values[i]
                    print(f"New best {monitor} value, saving model." if save else
                          f"No improvement over previous best {monitor} value, not saving model.")
                if save:
                    self.save(save_dir, saver, tags=save_tags, name=save_name, include_global_step=True,
                              include_last_training_loss=True, include_metrics=True)
            self.best_training_loss = min(self.best_training_loss, self.training_loss)
            if evaluated:
                for i, name in enumerate(self.metric_names):
                    better = (self.metric_values[i] < self.best_metric_values[i]) if name == "mean_loss" else \
                        (self.metric_values[i] > self.best_metric_values[i])
                    if better:
                        self.best_metric_values[i] = self.metric_values[i]

    def _evaluate(self, eval_dataset, num_batches, description="Running evaluation"):
        from tqdm import trange
        from .. import runtime
        if eval_dataset == "val":
            if self._val_iter is None:
                raise ValueError("no val_dataset")
            it = "_val_iter"
        else:
            it = "_train_iter"
        self._reset_metrics()
        show = (self.dist is None) or self.dist.get_rank() == 0
        tr = trange(num_batches, file=sys.stdout, disable=not show)
        tr.set_description(description)
        ex_u8 = None
        for _ in tr:
            images, labels = self._next(it)
            images = self.native._images(images)
            labels = self._targets(labels)
            if ex_u8 is None:
                ex_u8 = self.native.executor(images.dtype == self._torch.uint8, inference=True)
            probs = ex_u8.forward(self.native.params, images)
            runtime.batch_metrics(probs, labels, None, self._accum)
        self.metric_values = self._metric_values()

    def evaluate(self, eval_dataset="val", num_batches=1, dataset="val"):
        """Mean loss and accuracy over num_batches batches of the train or
        val stream (:708-750)."""
        if eval_dataset not in ("train", "val"):
            raise ValueError("`dataset` must be either 'train' or 'val'.")
        self._initialize_metrics()
        self._evaluate(eval_dataset, num_batches, "Running evaluation")
        self.eval_dataset = eval_dataset
        return dict(zip(self.metric_names, self.metric_values))

    def predict(self, images, argmax=True):
        probs = self.native.predict(images)
        return probs.argmax(axis=-1) if argmax else probs

    # -- persistence -----------------------------------------------------------------
    def save(self, model_save_dir, saver, tags=["default"], name=None, include_global_step=True,
             include_last_training_loss=True, include_metrics=True, force_save=False):
        """Writes <dir>/<model name>/variables.npz (Keras-order weights +
        Adam state) and state.json (global step, metrics) on rank 0; the
        directory name follows the reference's pattern (:781-858)."""
        if not self.variables_updated and not force_save:
            print("Abort: Nothing to save, no training has been performed since the model was last saved.")
            return None
        if saver not in ("saved_model", "train_saver"):
            raise ValueError("Unexpected value for `saver`: Can be either 'saved_model' or 'train_saver', "
                             f"but received '{saver}'.")
        if self.training_loss is None:
            include_last_training_loss = False
        model_name = "saved_model"
        if name:
            model_name += "_" + name
        if include_global_step:
            model_name += f"_(globalstep-{self.g_step})"
        if include_last_training_loss:
            model_name += f"_(trainloss-{self.training_loss:.4f})"
        if include_metrics:
            model_name += "_(eval_on_val_dataset)" if self.eval_dataset == "val" else "_(eval_on_train_dataset)"
            for n, v in zip(self.metric_names, self.metric_values):
                model_name += f"_({n}-{v:.4f})"
        if not (include_global_step or include_last_training_loss or include_metrics) and not name:
            model_name += f"_{time.time()}"
        path = os.path.join(model_save_dir, model_name)
        if (self.dist is None) or self.dist.get_rank() == 0:
            pathlib.Path(path).mkdir(parents=True, exist_ok=True)
            self.native.pull_weights()
            arrays = {f"w{i:05d}": w for i, w in enumerate(self.model.get_weights())}
            if self.native.m is not None:
                arrays["adam_m"] = self.native.m.cpu().numpy()
                arrays["adam_v"] = self.native.v.cpu().numpy()
            np.savez(os.path.join(path, "variables.npz"), **arrays)
            with open(os.path.join(path, "state.json"), "w") as f:
                json.dump({"global_step": self.g_step, "adam_step": self.native.step, "saver": saver,
                           "tags": list(tags), "metrics": dict(zip(self.metric_names, self.metric_values))}, f)
        self.variables_updated = False
        return path

    def load_variables(self, path):
        """Restore weights (+ Adam state when present) saved by save()."""
        torch = self._torch
        d = path if os.path.isdir(path) else os.path.dirname(path)
        with np.load(os.path.join(d, "variables.npz"), allow_pickle=False) as f:
            ws = [f[k] for k in sorted(k for k in f.files if k.startswith("w"))]
            self.model.set_weights(ws)
            if "adam_m" in f.files:
                self.native.m = torch.from_numpy(f["adam_m"]).to(self.native.device)
                self.native.v = torch.from_numpy(f["adam_v"]).to(self.native.device)
        st = os.path.join(d, "state.json")
        if os.path.exists(st):
            with open(st) as f:
                s = json.load(f)
            self.g_step = int(s.get("global_step", self.g_step))
            self.native.step = int(s.get("adam_step", self.native.step))

    def close(self):
        for f in (getattr(self, "csv_file_train", None), getattr(self, "csv_file_val", None)):
            if f is not None:
                f.close()
