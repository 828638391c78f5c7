"""Sampling drivers and MCEM of the reference's experiments/utils_training.py on the MI355X engine.

Same functions, signatures, schedule and sample bookkeeping as the reference:
  regression_train / classification_train          utils_training.py:11-172
  MCEM_sampler_UCI / MCEM_sampler_classification    :174-336
  MCEM_Q_maximizer                                  :339-358
  MCEM / MCEM_windows / MCEM_increasing_windows     :360-473

Per epoch the reference runs precond_update, then one sgmcmc_update per minibatch with lr_0 and
T = 0 during burn-in and lr_0 * cyclical_step_rate(...)^2, T = 1 afterwards, scoring the test set at
the end of each cycle.  Here an epoch of steps is a few replays of one captured hipGraph (at most
EPOCH_GRAPH_STEPS steps each): minibatches are drawn
on the device (per-epoch permutation, drop remainder), and the burn-in / cosine schedule and the
cycle-head momentum resampling are evaluated inside the update kernel from the device step counter
(DGPRF_SCHED_CYCLICAL, the same float32 formula as utils.py:49-73 with min_value = 0).  The host
only launches graphs and scores samples.  random_fixed=False layers redraw z every step on the
device (Philox keyed on the step counter).  Full-Bayes sampling of such a model, and datasets that
are not DeviceDatasets, take the reference's per-batch loop instead.

Deliberate differences: samples are COPIES of W (the reference appends the
live variables, so every stored "sample" aliases the current W; set REFERENCE_SAMPLE_ALIASING = True
to reproduce that), and the test set is scored in a fixed order (utils_dataset.load_arrays).
"""
import numpy as np
import torch

from experiments.utils_dataset import (DeviceDataset, download_UCI_data_info, load_UCI_dataset,
                                       load_arrays, load_tf_dataset, normalize_MNIST)
from utils import cyclical_step_rate

REFERENCE_SAMPLE_ALIASING = False
# steps per captured graph of an epoch: config 2's 5,000-step epoch as one 5,000-step graph ran
# 30.9 us/step against 27.9 for replays of a 100-step graph (bench.py `driver`, same box)
EPOCH_GRAPH_STEPS = 100


def _store_W(model):
    if REFERENCE_SAMPLE_ALIASING:
        return model.W_mcmc
    return [W.detach().clone() for W in model.W_mcmc]


def _graph_ok(model, ds_train, full_bayesian=False):
    return (isinstance(ds_train, DeviceDataset) and ds_train.drop_remainder and
            ds_train.batch_size is not None and
            (not full_bayesian or
             all(model.BNN.layers[2 * l].random_fixed for l in range(model.n_hidden_layers))))


def _run_epochs(model, ds_train, ds_M, data_size, batch_size, lr_0, momentum_decay,
                full_bayesian, precond_type, K_batches, second_moment_centered,
                resample_in_cycle_head, total_epochs, start_sampling_epoch, epochs_per_cycle,
                on_sample, on_epoch_end=None):
    """The epoch/batch loop shared by every driver (utils_training.py:41-70, 205-233)."""
    iterations_per_epoch = ds_train.num_batches() if isinstance(ds_train, DeviceDataset) \
        else sum(1 for _ in ds_train)
    cycle_length = epochs_per_cycle * iterations_per_epoch
    graph = _graph_ok(model, ds_train, full_bayesian)
    if graph:
        # schedule clock: the device step counter at the driver's first step is step_index 1 of
        # the burn-in; sampling starts start_sampling_epoch epochs later
        t0 = int(model._engine.step_ctr.item())
    for epoch in range(total_epochs):
        model.precond_update(ds_M, data_size, K_batches=K_batches, full_bayesian=full_bayesian,
                             precond_type=precond_type,
                             second_moment_centered=second_moment_centered)
        if graph:
            # the epoch as replays of one graph of at most EPOCH_GRAPH_STEPS steps (the schedule
            # and minibatch position come from the device step counter, so a graph replays
            # anywhere in the epoch)
            model.run_sgmcmc(ds_train.X, ds_train.Y, data_size, iterations_per_epoch,
                             batch_size=ds_train.batch_size, lr=lr_0,
                             momentum_decay=momentum_decay, temperature=1.,
                             steps_per_graph=min(iterations_per_epoch, EPOCH_GRAPH_STEPS),
                             perm_seed=ds_train.seed,
                             schedule='cyclical',
                             start_step=t0 + start_sampling_epoch * iterations_per_epoch,
                             cycle_length=cycle_length,
                             resample_in_cycle_head=resample_in_cycle_head,
                             full_bayesian=full_bayesian)
        else:
            batch_index = 0
            for img_batch, label_batch in ds_train:
                batch_index = batch_index + 1
                if epoch < start_sampling_epoch:
                    model.sgmcmc_update(img_batch, label_batch, data_size, lr=lr_0,
                                        momentum_decay=momentum_decay,
                                        full_bayesian=full_bayesian, resample_moments=False,
                                        temperature=0.)
                else:
                    step_index = (epoch - start_sampling_epoch) * iterations_per_epoch + \
                        batch_index
                    step_rate, _ = cyclical_step_rate(step_index, cycle_length,
                                                      schedule='cosine', min_value=0.)
                    lr = lr_0 * (step_rate ** 2)
                    is_new_cycle = bool(resample_in_cycle_head) and \
                        (step_index % cycle_length == 1)
                    model.sgmcmc_update(img_batch, label_batch, data_size, lr=lr,
                                        momentum_decay=momentum_decay,
                                        full_bayesian=full_bayesian,
                                        resample_moments=is_new_cycle, temperature=1.)
        # is_end of cyclical_step_rate falls on the last batch of every epochs_per_cycle-th
        # sampling epoch (cycle_length is a whole number of epochs)
        if epoch >= start_sampling_epoch and \
                (epoch - start_sampling_epoch + 1) % epochs_per_cycle == 0:
            step_index = (epoch - start_sampling_epoch + 1) * iterations_per_epoch
            step_rate, is_end = cyclical_step_rate(step_index, cycle_length, schedule='cosine',
                                                   min_value=0.)
            assert is_end
            on_sample(epoch, lr_0 * (step_rate ** 2))
        if on_epoch_end is not None:
            on_epoch_end(epoch)


def _summary_regression(log_p, mse):
    log_p = torch.stack(log_p, dim=0)  # [S, N]
    mse = torch.stack(mse, dim=0)      # [S, N]
    n_models = mse.shape[0]
    predict_log_p = torch.logsumexp(log_p, dim=0) - np.log(float(n_models))
    return log_p, mse, n_models, float(torch.mean(predict_log_p)), \
        float(torch.sqrt(torch.mean(mse)))


def _summary_classification(log_p, acc):
    log_p = torch.stack(log_p, dim=0)  # [S, N]
    acc = torch.stack([torch.as_tensor(a, dtype=torch.float32) for a in acc], dim=0)  # [S]
    n_models = acc.shape[0]
    predict_log_p = torch.logsumexp(log_p, dim=0) - np.log(float(n_models))
    return log_p, acc, n_models, float(torch.mean(predict_log_p)), float(torch.mean(acc))


def _regression_data(dataset_name, batch_size, data_dir, data):
    """(ds_train, ds_test, train_size, batch_size, Y_std) — utils_training.py:19-31.
    `data` = (X, Y, Xs, Ys[, Y_std]) arrays bypass the CSV loader."""
    if data is None:
        _, _, _, _, _, _, Y_std = download_UCI_data_info(dataset_name, data_path=data_dir)
        Y_std = float(Y_std[0])
        ds_train, ds_test, train_shape, test_shape = load_UCI_dataset(
            dataset_name, batch_size=batch_size, data_dir=data_dir)
    else:
        X, Y, Xs, Ys = data[:4]
        Y_std = float(data[4]) if len(data) > 4 else 1.0
        ds_train, ds_test, train_shape, test_shape = load_arrays(X, Y, Xs, Ys, batch_size)
    train_size = train_shape[0]
    if train_size - train_size % batch_size == 0:  # batch size > train size
        print("Training size is 0 after remainder dropping! Using the whole data as one batch! ")
        ds_train = ds_train.batch(train_size, drop_remainder=False)
        batch_size = train_size
    print(f"Training size is {train_size - train_size % batch_size} after remainder dropping. ")
    return ds_train, ds_test, train_size, batch_size, Y_std


def _check_precond(precond_type, K_batches, second_moment_centered):
    if precond_type != 'identity' and K_batches is None and second_moment_centered is None:
        raise ValueError("Args K_batches or second_moment_centered shouldn't be None!")


def regression_train(model, dataset_name='boston', batch_size=200, data_dir='./data/',
                     lr_0=0.01, momentum_decay=0.9, full_bayesian=True,
                     precond_type='identity', K_batches=None, second_moment_centered=None,
                     resample_in_cycle_head=False,
                     total_epochs=5000, start_sampling_epoch=2000, epochs_per_cycle=50,
                     print_epoch_cycle=100, data=None):
    """utils_training.py:11-88 -> (log_p [S, N_test], mse [S, N_test])."""
    _check_precond(precond_type, K_batches, second_moment_centered)
    ds_train, ds_test, train_size, batch_size, Y_std = _regression_data(
        dataset_name, batch_size, data_dir, data)
    log_p, mse = [], []
    state = {"k": 0}

    def on_sample(epoch, lr):
        test_log_p, test_se = model.eval_log_likelihood_and_se(ds_test)
        log_p.append(test_log_p - np.log(Y_std))  # restore via Y_std
        mse.append(test_se * Y_std ** 2.)
        state["k"] += 1
        print('#' * 20, f'Sample No.{state["k"]} at Epoch {epoch} ', f"lr = {lr}", '#' * 20)

    def on_epoch_end(epoch):
        if (epoch + 1) % print_epoch_cycle == 0:
            _print_regression(model, ds_train, ds_test, Y_std, f"Epoch: {epoch}")

    _run_epochs(model, ds_train, ds_train, train_size, batch_size, lr_0, momentum_decay,
                full_bayesian, precond_type, K_batches, second_moment_centered,
                resample_in_cycle_head, total_epochs, start_sampling_epoch, epochs_per_cycle,
                on_sample, on_epoch_end)
    log_p, mse, n_models, ll, rmse = _summary_regression(log_p, mse)
    print(f"Dataset: {dataset_name}, Number of sampled models: {n_models} ")
    print(f"Test Log Likelihood of all sampled models: {ll}")
    print(f"Test Root MSE of all sampled models: {rmse}")
    return log_p, mse


def _print_regression(model, ds_train, ds_test, Y_std, head):
    train_log_p, train_se = model.eval_log_likelihood_and_se(ds_train)
    test_log_p, test_se = model.eval_log_likelihood_and_se(ds_test)
    print(head)
    print(f"Mean Log Likelihood -- train: {float(torch.mean(train_log_p)) - np.log(Y_std)}, "
          f"-- test: {float(torch.mean(test_log_p)) - np.log(Y_std)} ")
    print(f"Root Mean Squared Error -- train: {float(torch.sqrt(torch.mean(train_se))) * Y_std}, "
          f"-- test: {float(torch.sqrt(torch.mean(test_se))) * Y_std} \n")


def _print_classification(model, ds_train, ds_test, head):
    train_log_p = model.eval_log_likelihood(ds_train)
    test_log_p = model.eval_log_likelihood(ds_test)
    print(head)
    print(f"Mean Log Likelihood -- train: {float(torch.mean(train_log_p))}, "
          f"-- test: {float(torch.mean(test_log_p))} ")
    print(f"Accuracy -- train: {float(model.eval_all_accuracy(ds_train))}, "
          f"-- test: {float(model.eval_all_accuracy(ds_test))} \n")


def _classification_data(dataset_name, batch_size, data_dir, data):
    if data is None:
        ds_train, ds_test, train_full_size, _ = load_tf_dataset(
            dataset_name, transform_fn=normalize_MNIST, batch_size=batch_size, data_dir=data_dir)
    else:
        X, Y, Xs, Ys = data[:4]
        ds_train, ds_test, tr_shape, _ = load_arrays(X, Y, Xs, Ys, batch_size)
        train_full_size = tr_shape[0]
    if train_full_size - train_full_size % batch_size == 0:
        print("Training size is 0 after remainder dropping! Using the whole data as one batch! ")
        ds_train = ds_train.batch(train_full_size, drop_remainder=False)
        batch_size = train_full_size
    print(f"Training size is {train_full_size - train_full_size % batch_size} after remainder "
          f"dropping. ")
    return ds_train, ds_test, train_full_size, batch_size


def classification_train(model, dataset_name='mnist', batch_size=200,
                         data_dir='./tensorflow_datasets/', lr_0=0.01, momentum_decay=0.9,
                         full_bayesian=True, precond_type='identity', K_batches=None,
                         second_moment_centered=None, resample_in_cycle_head=False,
                         total_epochs=5000, start_sampling_epoch=2000, epochs_per_cycle=50,
                         print_epoch_cycle=100, data=None):
    """utils_training.py:90-172 -> (log_p [S, N_test], acc [S])."""
    _check_precond(precond_type, K_batches, second_moment_centered)
    ds_train, ds_test, train_full_size, batch_size = _classification_data(
        dataset_name, batch_size, data_dir, data)
    log_p, acc = [], []
    state = {"k": 0}

    def on_sample(epoch, lr):
        log_p.append(model.eval_log_likelihood(ds_test))
        acc.append(model.eval_all_accuracy(ds_test))
        state["k"] += 1
        print('#' * 20, f'Sample No.{state["k"]} at Epoch {epoch} ', f"lr = {lr}", '#' * 20)

    def on_epoch_end(epoch):
        if (epoch + 1) % print_epoch_cycle == 0:
            _print_classification(model, ds_train, ds_test, f"Epoch: {epoch}")

    _run_epochs(model, ds_train, ds_train, train_full_size, batch_size, lr_0, momentum_decay,
                full_bayesian, precond_type, K_batches, second_moment_centered,
                resample_in_cycle_head, total_epochs, start_sampling_epoch, epochs_per_cycle,
                on_sample, on_epoch_end)
    log_p, acc, n_models, ll, macc = _summary_classification(log_p, acc)
    print(f"Dataset: {dataset_name}, Number of sampled models: {n_models} ")
    print(f"Test Log Likelihood of all sampled models: {ll}")
    print(f"Test Mean Acc of all sampled models: {macc}")
    return log_p, acc


def MCEM_sampler_UCI(model, dataset_name='boston', batch_size=200, data_dir='./data/',
                     lr_0=0.01, momentum_decay=0.9,
                     precond_type='identity', K_batches=None, second_moment_centered=None,
                     resample_in_cycle_head=True, start_sampling_epoch=2000, epochs_per_cycle=50,
                     data=None):
    """utils_training.py:174-254: returns sampler(num_samples, print_epoch_cycle) ->
    (W_samples, log_p [S, N], mse [S, N]); W-only sampling (full_bayesian=False)."""
    _check_precond(precond_type, K_batches, second_moment_centered)
    ds_train, ds_test, train_size, batch_size, Y_std = _regression_data(
        dataset_name, batch_size, data_dir, data)

    def sampler(num_samples=100, print_epoch_cycle=100):
        total_epochs = start_sampling_epoch + num_samples * epochs_per_cycle
        W_samples, log_p, mse = [], [], []
        state = {"k": 0}

        def on_sample(epoch, lr):
            state["k"] += 1
            W_samples.append(_store_W(model))
            print('#' * 20, f'Sample No.{state["k"]} at Epoch {epoch} ', f"lr = {lr}", '#' * 20)
            test_log_p, test_se = model.eval_log_likelihood_and_se(ds_test)
            log_p.append(test_log_p - np.log(Y_std))
            mse.append(test_se * Y_std ** 2)

        def on_epoch_end(epoch):
            if (epoch + 1) % print_epoch_cycle == 0:
                _print_regression(model, ds_train, ds_test, Y_std, f"Sampling Epoch: {epoch}")

        _run_epochs(model, ds_train, ds_train, train_size, batch_size, lr_0, momentum_decay,
                    False, precond_type, K_batches, second_moment_centered,
                    resample_in_cycle_head, total_epochs, start_sampling_epoch, epochs_per_cycle,
                    on_sample, on_epoch_end)
        log_p, mse, n_models, ll, rmse = _summary_regression(log_p, mse)
        print("*" * 20, f" Dataset: {dataset_name} -- End of Sampling ", "*" * 20)
        print(f"Number of sampled models: {n_models} ")
        print(f"Test Log Likelihood of all sampled models: {ll}")
        print(f"Test Root MSE of all sampled models: {rmse}")
        print("*" * 70, "\n")
        return W_samples, log_p, mse

    sampler.ds_train = ds_train
    return sampler


def MCEM_sampler_classification(model, dataset_name='boston', batch_size=200,
                                data_dir='./tensorflow_datasets/', lr_0=0.01, momentum_decay=0.9,
                                precond_type='identity', K_batches=None,
                                second_moment_centered=None, resample_in_cycle_head=True,
                                start_sampling_epoch=2000, epochs_per_cycle=50, data=None):
    """utils_training.py:256-336: sampler(...) -> (W_samples, log_p [S, N], acc [S])."""
    _check_precond(precond_type, K_batches, second_moment_centered)
    ds_train, ds_test, train_full_size, batch_size = _classification_data(
        dataset_name, batch_size, data_dir, data)

    def sampler(num_samples=100, print_epoch_cycle=100):
        total_epochs = start_sampling_epoch + num_samples * epochs_per_cycle
        W_samples, log_p, acc = [], [], []
        state = {"k": 0}

        def on_sample(epoch, lr):
            state["k"] += 1
            W_samples.append(_store_W(model))
            log_p.append(model.eval_log_likelihood(ds_test))
            acc.append(model.eval_all_accuracy(ds_test))
            print('#' * 20, f'Sample No.{state["k"]} at Epoch {epoch} ', f"lr = {lr}", '#' * 20)

        def on_epoch_end(epoch):
            if (epoch + 1) % print_epoch_cycle == 0:
                _print_classification(model, ds_train, ds_test, f"Epoch: {epoch}")

        _run_epochs(model, ds_train, ds_train, train_full_size, batch_size, lr_0,
                    momentum_decay, False, precond_type, K_batches, second_moment_centered,
                    resample_in_cycle_head, total_epochs, start_sampling_epoch, epochs_per_cycle,
                    on_sample, on_epoch_end)
        log_p, acc, n_models, ll, macc = _summary_classification(log_p, acc)
        print("*" * 20, f" Dataset: {dataset_name} -- End of Sampling ", "*" * 20)
        print(f"Number of sampled models: {n_models} ")
        print(f"Test Log Likelihood of all sampled models: {ll}")
        print(f"Test Mean Acc of all sampled models: {macc}")
        print("*" * 70, "\n")
        return W_samples, log_p, acc

    sampler.ds_train = ds_train
    return sampler


def MCEM_Q_maximizer(model, data_size, optimizer):
    """utils_training.py:339-358: maximizer(W_samples, X_batch, Y_batch) takes one optimizer
    step on -Q over Omega_hyperparams + Likelihood_hyperparams.  The gradient is the device
    backward (model.Q_and_hyper_grads), not an autodiff tape."""
    def maximizer(W_samples, X_batch, Y_batch):
        Q, grads = model.Q_and_hyper_grads(W_samples, X_batch, Y_batch, data_size)
        print("*" * 70)
        print(f"Q function is {float(Q)} averaged by {len(W_samples)} samples.")
        print("*" * 70, "\n")
        optimizer.apply_gradients(zip(grads, model.hyper_variables()))
        return Q
    return maximizer


def MCEM(sampler_EM, maximizer, sampler_fixing_hyper, total_EM_steps, ds_train,
         num_samples_EM=100, num_samples_fixing_hyper=200,
         print_epoch_cycle_EM=100, print_epoch_cycle_fixing=100):
    """utils_training.py:360-379 -> (log_p, mse_or_acc) of the final fixed-hyper sampling."""
    em_step = 0
    for x_batch, y_batch in ds_train.repeat():
        em_step += 1
        print("#" * 15, f"EM step {em_step} of total {total_EM_steps} steps. E Step: ", "#" * 15)
        W_samples, _, _ = sampler_EM(num_samples=num_samples_EM,
                                     print_epoch_cycle=print_epoch_cycle_EM)
        print("#" * 15, f"EM step {em_step} of total {total_EM_steps} steps, M Step: ", "#" * 15)
        maximizer(W_samples, x_batch, y_batch)
        if em_step == total_EM_steps:
            break
    print("#" * 15, f"After {total_EM_steps} EM steps, fixing hyperparams and sample from "
          "posterior.", "#" * 15)
    _, log_p, mse_or_acc = sampler_fixing_hyper(num_samples=num_samples_fixing_hyper,
                                                print_epoch_cycle=print_epoch_cycle_fixing)
    return log_p, mse_or_acc


def _window_em(sampler_EM, maximizer, sampler_fixing_hyper, total_EM_steps, ds_train,
               num_samples_fixing_hyper, window_size, print_epoch_cycle_EM,
               print_epoch_cycle_fixing, rank1_is_acc):
    """MCEM_windows / MCEM_increasing_windows (utils_training.py:381-473): one sample per E step
    into a sliding window, M step on one uniformly chosen window member."""
    W_window, log_p_window, m_window = [], None, None
    em_step = 0
    for x_batch, y_batch in ds_train.repeat():
        em_step += 1
        print("#" * 15, f"EM step {em_step} of total {total_EM_steps} steps. E Step: ", "#" * 15)
        W_samples, log_p, m = sampler_EM(num_samples=1, print_epoch_cycle=print_epoch_cycle_EM)
        W_window.extend(W_samples)
        if len(W_window) == 1:
            log_p_window, m_window = log_p, m
        elif len(W_window) <= window_size:
            log_p_window = torch.cat([log_p_window, log_p], dim=0)
            m_window = torch.cat([m_window, m], dim=0)
        else:
            W_window = W_window[-window_size:]
            log_p_window = torch.cat([log_p_window, log_p], dim=0)[1:]
            m_window = torch.cat([m_window, m], dim=0)[1:]
        n_models = m_window.shape[0]
        ll = float(torch.mean(torch.logsumexp(log_p_window, dim=0) - np.log(float(n_models))))
        print("*" * 20, " End of E step ", "*" * 20)
        print(f"Number of all sampled models in window: {n_models} ")
        print(f"Test Log Likelihood of all models in window: {ll}")
        if m_window.dim() == 1 and rank1_is_acc:
            print(f"Test Mean Acc of all models in window: {float(torch.mean(m_window))}\n")
        else:
            print(f"Test Root MSE of all models in window: "
                  f"{float(torch.sqrt(torch.mean(m_window)))}\n")
        print("#" * 15, f"EM step {em_step} of total {total_EM_steps} steps, M Step: ", "#" * 15)
        i = np.random.randint(len(W_window))
        maximizer([W_window[i]], x_batch, y_batch)
        if em_step == total_EM_steps:
            break
    print("#" * 15, f"After {total_EM_steps} EM steps, fixing hyperparams and sample from "
          "posterior.", "#" * 15)
    _, log_p, m = sampler_fixing_hyper(num_samples=num_samples_fixing_hyper,
                                       print_epoch_cycle=print_epoch_cycle_fixing)
    return log_p, m


def MCEM_windows(sampler_EM, maximizer, sampler_fixing_hyper, total_EM_steps, ds_train,
                 num_samples_fixing_hyper=200, window_size=300,
                 print_epoch_cycle_EM=100, print_epoch_cycle_fixing=100):
    """utils_training.py:381-428."""
    return _window_em(sampler_EM, maximizer, sampler_fixing_hyper, total_EM_steps, ds_train,
                      num_samples_fixing_hyper, window_size, print_epoch_cycle_EM,
                      print_epoch_cycle_fixing, rank1_is_acc=True)


def MCEM_increasing_windows(sampler_EM, maximizer, sampler_fixing_hyper, total_EM_steps,
                            ds_train, num_samples_fixing_hyper=200, window_size=300,
                            print_epoch_cycle_EM=100, print_epoch_cycle_fixing=100):
    """utils_training.py:430-473 (regression: the window metric is always an MSE matrix)."""
    return _window_em(sampler_EM, maximizer, sampler_fixing_hyper, total_EM_steps, ds_train,
                      num_samples_fixing_hyper, window_size, print_epoch_cycle_EM,
                      print_epoch_cycle_fixing, rank1_is_acc=False)
