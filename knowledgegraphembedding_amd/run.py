#!/usr/bin/python3
"""Training / evaluation CLI — the reference's codes/run.py, flag for flag.

    python -m knowledgegraphembedding_amd.run --do_train --cuda --do_valid --do_test \
        --data_path data/FB15k --model RotatE -n 256 -b 1024 -d 1000 -g 24.0 -a 1.0 -adv \
        -lr 0.0001 --max_steps 150000 -save models/RotatE_FB15k_0 --test_batch_size 16 -de

Differences from the reference, all on the execution side:
  * compute runs on the GPU through libkge_hip.so (there is no CPU path;
    --cuda is implied when a GPU is present and required otherwise);
  * the optimizer is KGEAdam (torch.optim.Adam's update, fused), state-dict
    compatible with the reference's checkpoints;
  * under torchrun (WORLD_SIZE > 1) every rank trains on its own -b batch and
    gradients are all-reduced over RCCL (knowledgegraphembedding_amd.distributed);
    rank 0 logs, validates and saves.
"""
from __future__ import absolute_import, division, print_function

import argparse
import json
import logging
import os

import numpy as np
import torch
from torch.utils.data import DataLoader

from .dataloader import BidirectionalOneShotIterator, RankShardSampler, TrainDataset
from .model import KGEModel
from .optim import KGEAdam


_FLAG = dict(action='store_true')

# The reference's command line (codes/run.py:24-72): the same flags, short
# forms, defaults and types, plus two extensions at the end.
_CLI = (
    (('--cuda',), dict(_FLAG, help='compute on the GPU (implied: there is no CPU path)')),
    (('--do_train',), _FLAG),
    (('--do_valid',), _FLAG),
    (('--do_test',), _FLAG),
    (('--evaluate_train',), dict(_FLAG, help='also rank the training triples')),
    (('--countries',), dict(_FLAG, help='Countries S1/S2/S3: AUC-PR over the regions')),
    (('--regions',), dict(type=int, nargs='+', default=None, help='filled in from regions.list, not by hand')),
    (('--data_path',), dict(type=str, default=None)),
    (('--model',), dict(default='TransE', type=str)),
    (('-de', '--double_entity_embedding'), _FLAG),
    (('-dr', '--double_relation_embedding'), _FLAG),
    (('-n', '--negative_sample_size'), dict(default=128, type=int)),
    (('-d', '--hidden_dim'), dict(default=500, type=int)),
    (('-g', '--gamma'), dict(default=12.0, type=float)),
    (('-adv', '--negative_adversarial_sampling'), _FLAG),
    (('-a', '--adversarial_temperature'), dict(default=1.0, type=float)),
    (('-b', '--batch_size'), dict(default=1024, type=int)),
    (('-r', '--regularization'), dict(default=0.0, type=float)),
    (('--test_batch_size',), dict(default=4, type=int, help='queries per ranking batch')),
    (('--uni_weight',), dict(_FLAG, help='plain means instead of the word2vec-style subsampling weights')),
    (('-lr', '--learning_rate'), dict(default=0.0001, type=float)),
    (('-cpu', '--cpu_num'), dict(default=10, type=int)),
    (('-init', '--init_checkpoint'), dict(default=None, type=str)),
    (('-save', '--save_path'), dict(default=None, type=str)),
    (('--max_steps',), dict(default=100000, type=int)),
    (('--warm_up_steps',), dict(default=None, type=int)),
    (('--save_checkpoint_steps',), dict(default=10000, type=int)),
    (('--valid_steps',), dict(default=10000, type=int)),
    (('--log_steps',), dict(default=100, type=int, help='training log interval in steps')),
    (('--test_log_steps',), dict(default=1000, type=int, help='evaluation log interval in batches')),
    (('--nentity',), dict(type=int, default=0, help='filled in from entities.dict, not by hand')),
    (('--nrelation',), dict(type=int, default=0, help='filled in from relations.dict, not by hand')),
    (('--row_partition',), dict(_FLAG, help='multi-GPU only: each rank owns 1/world of the entity rows and '
                                            'their Adam state (partition.py; KGE_PART_EXCHANGE=factors|grads|'
                                            'queries, "queries" keeps only the shard on each rank and ships q '
                                            'vectors instead of rows)')),
    (('--device_sampler',), dict(_FLAG, help='build training batches on the GPU (sampler.py) instead of the '
                                             'CPU TrainDataset workers: same sampling semantics, a different '
                                             'random stream')),
)

# what -init restores from the checkpoint's config.json (codes/run.py:75-90);
# data_path only when the command line gives none
_RESTORED = ('countries', 'model', 'double_entity_embedding', 'double_relation_embedding', 'hidden_dim',
             'test_batch_size')


def parse_args(args=None):
    cli = argparse.ArgumentParser(description='Training and Testing Knowledge Graph Embedding Models',
                                  usage='train.py [<args>] [-h | --help]')
    for names, options in _CLI:
        cli.add_argument(*names, **options)
    return cli.parse_args(args)


def override_config(args):
    '''Restore the model/data configuration of -init (run.py:75-90).'''
    with open(os.path.join(args.init_checkpoint, 'config.json')) as f:
        saved = json.load(f)
    for key in _RESTORED:
        setattr(args, key, saved[key])
    if args.data_path is None:
        args.data_path = saved['data_path']


def _json_args(args):
    return {k: v for k, v in vars(args).items() if not k.startswith('dp_')}


def save_model(model, optimizer, save_variable_list, args, optimizer_state=None):
    '''config.json + checkpoint + entity/relation_embedding.npy (run.py:93-120).
    `optimizer_state` overrides optimizer.state_dict() (the row-partitioned
    trainer passes its state gathered to the full-table layout).'''
    with open(os.path.join(args.save_path, 'config.json'), 'w') as fjson:
        json.dump(_json_args(args), fjson)
    torch.save({
        **save_variable_list,
        'model_state_dict': model.state_dict(),
        'optimizer_state_dict': optimizer.state_dict() if optimizer_state is None else optimizer_state},
        os.path.join(args.save_path, 'checkpoint')
    )
    np.save(os.path.join(args.save_path, 'entity_embedding'), model.entity_embedding.detach().cpu().numpy())
    np.save(os.path.join(args.save_path, 'relation_embedding'), model.relation_embedding.detach().cpu().numpy())


def _tsv(file_path):
    with open(file_path) as f:
        return [line.strip().split('\t') for line in f]


def read_triple(file_path, entity2id, relation2id):
    '''Triples mapped to ids (run.py:123-132).'''
    return [(entity2id[h], relation2id[r], entity2id[t]) for h, r, t in _tsv(file_path)]


def read_dict(file_path):
    '''name → id of entities.dict / relations.dict (lines "<id>\\t<name>").'''
    return {name: int(eid) for eid, name in _tsv(file_path)}


def shared_seed(group=None) -> int:
    """A sampler seed that is the same on every rank: rank 0's torch seed,
    broadcast (a per-rank seed would make the ranks' shards of an epoch
    overlap or skip positives, undetected)."""
    import torch.distributed as dist
    seed = [int(torch.initial_seed()) % (1 << 31)]
    if dist.is_available() and dist.is_initialized():
        dist.broadcast_object_list(seed, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group)
    return int(seed[0])


WORKER_START_METHOD = "forkserver"


def worker_context(method=None):
    """The multiprocessing context of the host DataLoader workers.

    The reference's workers are fork()ed from its training process
    (run.py:246-260, torch's default).  Here that process holds a HIP
    context — and, under torchrun, an RCCL communicator — whose runtime
    threads (ROCr's async-event thread, RCCL's proxy / bootstrap threads,
    c10d's watchdog and store threads) may hold their locks at the moment of
    the fork, and whose heap still holds device-side objects — CUDA / pinned
    tensors, events, communicator work items — in uncollected reference
    cycles.  A fork copies one thread and all of that memory: when the
    child's cyclic GC frees one of those objects, torch's caching allocators
    call into the HIP runtime of a process that no longer has one (its
    service threads did not survive the fork), or the child blocks on a lock
    a parent thread held — the worker never answers and the trainer waits on
    it forever (the round-4 GPU-suite hang: run.py's DataLoader forked from a
    pytest process after an RCCL group had been created and destroyed in it;
    DESIGN §12).  Workers therefore start from a "forkserver": a fresh
    interpreter launched (fork + exec, no GPU state) the first time a context
    is asked for — run.py asks before it initialises RCCL or the GPU — which
    forks every worker from its own clean state.  Worker seeding is
    DataLoader's own (base seed from the loader's generator, numpy seeded
    from it in the worker), so the batches are the reference's bit for bit
    (tests/test_run_shard.py compares them with fork-started workers)."""
    import multiprocessing as mp
    method = method or WORKER_START_METHOD
    ctx = mp.get_context(method)
    if method == "forkserver":
        from multiprocessing import forkserver
        if not getattr(worker_context, "_preloaded", False):
            # the workers' imports, once, in the server (each fork inherits them)
            ctx.set_forkserver_preload(["torch", "numpy", "knowledgegraphembedding_amd.dataloader"])
            worker_context._preloaded = True
        forkserver.ensure_running()
    return ctx


def make_train_iterator(args, train_triples, nentity, nrelation, rank=0, world=1, seed=None, start_method=None):
    """run.py:246-259's two DataLoaders and BidirectionalOneShotIterator.  One
    process: exactly the reference's (shuffle=True on torch's global
    generator).  Under data parallelism each rank gets a disjoint shard of
    every epoch's permutation (RankShardSampler, `seed` — shared_seed() by
    default — the same on all ranks) and its own generator, so its workers'
    numpy streams — the negatives — differ from the other ranks' too.
    Workers start from worker_context(start_method) (forkserver by default:
    never a fork of a process that holds GPU / RCCL state)."""
    if world > 1 and seed is None:
        seed = shared_seed(getattr(args, 'dp_group', None))
    ctx = worker_context(start_method)

    def loader(mode):
        ds = TrainDataset(train_triples, nentity, nrelation, args.negative_sample_size, mode)
        kw = dict(batch_size=args.batch_size, num_workers=max(1, args.cpu_num // 2),
                  collate_fn=TrainDataset.collate_fn, multiprocessing_context=ctx)
        if world <= 1:
            return DataLoader(ds, shuffle=True, **kw)
        return DataLoader(ds, sampler=RankShardSampler(len(ds), rank, world, seed + (mode == 'tail-batch')),
                          generator=torch.Generator().manual_seed(seed + 7919 * (rank + 1)), **kw)

    return BidirectionalOneShotIterator(loader('head-batch'), loader('tail-batch'))


def set_logger(args, rank=0):
    '''Log to <save_path>/train.log (or test.log) and the console (run.py:135-156).'''
    if rank != 0:
        logging.basicConfig(level=logging.WARNING)
        return
    if args.do_train:
        log_file = os.path.join(args.save_path or args.init_checkpoint, 'train.log')
    else:
        log_file = os.path.join(args.save_path or args.init_checkpoint, 'test.log')
    for h in list(logging.getLogger('').handlers):
        logging.getLogger('').removeHandler(h)
    logging.basicConfig(format='%(asctime)s %(levelname)-8s %(message)s', level=logging.INFO,
                        datefmt='%Y-%m-%d %H:%M:%S', filename=log_file, filemode='w')
    console = logging.StreamHandler()
    console.setLevel(logging.INFO)
    console.setFormatter(logging.Formatter('%(asctime)s %(levelname)-8s %(message)s'))
    logging.getLogger('').addHandler(console)


def log_metrics(mode, step, metrics):
    for metric in metrics:
        logging.info('%s %s at step %d: %f' % (mode, metric, step, metrics[metric]))


def _init_distributed(args):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    args.dp_group = None
    if world <= 1:
        return 0
    import torch.distributed as dist
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group('nccl' if torch.cuda.is_available() else 'gloo')
    args.dp_group = dist.group.WORLD
    return dist.get_rank()


def main(args):
    if (not args.do_train) and (not args.do_valid) and (not args.do_test):
        raise ValueError('one of train/val/test mode must be choosed.')
    if args.init_checkpoint:
        override_config(args)
    elif args.data_path is None:
        raise ValueError('one of init_checkpoint/data_path must be choosed.')
    if args.do_train and args.save_path is None:
        raise ValueError('Where do you want to save your trained model?')
    if args.do_train and not getattr(args, 'device_sampler', False):
        worker_context()  # the DataLoader workers' server starts before RCCL / HIP exist in this process
    rank = _init_distributed(args)
    if args.save_path and not os.path.exists(args.save_path) and rank == 0:
        os.makedirs(args.save_path)
    set_logger(args, rank)

    if not torch.cuda.is_available():
        raise RuntimeError('knowledgegraphembedding_amd computes on MI355X (ROCm) only; no GPU is visible')
    if not args.cuda:
        logging.info('--cuda implied: knowledgegraphembedding_amd has no CPU compute path')
        args.cuda = True

    entity2id, relation2id = (read_dict(os.path.join(args.data_path, f + '.dict')) for f in ('entities', 'relations'))
    if args.countries:
        with open(os.path.join(args.data_path, 'regions.list')) as f:
            args.regions = [entity2id[name.strip()] for name in f]

    nentity, nrelation = len(entity2id), len(relation2id)
    args.nentity, args.nrelation = nentity, nrelation
    for line in ('Model: %s' % args.model, 'Data Path: %s' % args.data_path, '#entity: %d' % nentity,
                 '#relation: %d' % nrelation):
        logging.info(line)
    split = {}
    for name in ('train', 'valid', 'test'):
        split[name] = read_triple(os.path.join(args.data_path, name + '.txt'), entity2id, relation2id)
        logging.info('#%s: %d' % (name, len(split[name])))
    train_triples, valid_triples, test_triples = split['train'], split['valid'], split['test']
    all_true_triples = train_triples + valid_triples + test_triples

    kge_model = KGEModel(model_name=args.model, nentity=nentity, nrelation=nrelation, hidden_dim=args.hidden_dim,
                         gamma=args.gamma, double_entity_embedding=args.double_entity_embedding,
                         double_relation_embedding=args.double_relation_embedding)
    logging.info('Model Parameter Configuration:')
    for name, param in kge_model.named_parameters():
        logging.info('Parameter %s: %s, require_grad = %s' % (name, str(param.size()), str(param.requires_grad)))
    kge_model = kge_model.cuda()
    if args.dp_group is not None:
        # replicas start from rank 0's initialisation
        import torch.distributed as dist
        for p in kge_model.parameters():
            dist.broadcast(p.data, src=0)
    part = None
    owner = False
    if args.dp_group is not None:
        from .distributed import dp_exchange_mode
        owner = dp_exchange_mode(torch.distributed.get_world_size(args.dp_group),
                                 getattr(args, 'dp_exchange', None)) == "owner"
    if getattr(args, 'row_partition', False) and args.dp_group is None:
        logging.info('--row_partition ignored: one process (launch with torchrun for a partitioned table)')
    elif getattr(args, 'row_partition', False) or owner:
        # --row_partition: exchange KGE_PART_EXCHANGE ("factors": owner-computes
        # from the exchanged row factors; "grads": reduce-scatter of the dense
        # gradient); the data-parallel "owner" exchange is the former
        from .partition import EntityRowPartition
        exchange = os.environ.get('KGE_PART_EXCHANGE', 'factors') if getattr(args, 'row_partition', False) \
            else 'factors'
        part = EntityRowPartition(kge_model, args.dp_group, exchange=exchange)
        logging.info('Entity rows partitioned (%s exchange): rank %d owns [%d, %d)' % (exchange, rank, part.e0,
                                                                                        part.e1))

    def trainable():
        return part.parameters() if part is not None else filter(lambda p: p.requires_grad, kge_model.parameters())

    def optimizer_state():
        # collective under --row_partition: every rank calls it, rank 0 writes
        return part.gathered_optimizer_state_dict(optimizer) if part is not None else None

    def full_table(on: bool) -> None:
        # collective: query shipping keeps only shards; gather the whole table
        # for checkpoints / evaluation and drop it again (other modes: no-op)
        if part is not None:
            part.materialize() if on else part.release()

    world = 1 if args.dp_group is None else torch.distributed.get_world_size(args.dp_group)
    if args.do_train and getattr(args, 'device_sampler', False):
        from .sampler import DeviceTrainIterator
        train_iterator = DeviceTrainIterator(train_triples, nentity, nrelation, args.negative_sample_size,
                                             args.batch_size, kge_model.entity_embedding.device,
                                             seed=torch.initial_seed() + rank, rank=rank, world=world,
                                             perm_seed=shared_seed(args.dp_group) if world > 1 else None)
    elif args.do_train:
        train_iterator = make_train_iterator(args, train_triples, nentity, nrelation, rank, world)
    if args.do_train:
        current_learning_rate = args.learning_rate
        optimizer = KGEAdam(trainable(), lr=current_learning_rate)
        warm_up_steps = args.warm_up_steps if args.warm_up_steps else args.max_steps // 2

    if args.init_checkpoint:
        logging.info('Loading checkpoint %s...' % args.init_checkpoint)
        checkpoint = torch.load(os.path.join(args.init_checkpoint, 'checkpoint'), map_location='cpu',
                                weights_only=True)
        init_step = checkpoint['step']
        full_table(True)
        kge_model.load_state_dict(checkpoint['model_state_dict'])
        if part is not None:
            part.reload_from_replica()
        full_table(False)
        if args.do_train:
            current_learning_rate = checkpoint['current_learning_rate']
            warm_up_steps = checkpoint['warm_up_steps']
            if part is not None:
                part.load_optimizer_state_dict(optimizer, checkpoint['optimizer_state_dict'])
            else:
                optimizer.load_state_dict(checkpoint['optimizer_state_dict'])
    else:
        logging.info('Ramdomly Initializing %s Model...' % args.model)
        init_step = 0

    step = init_step
    # the reference's start-up lines, verbatim (negative_adversarial_sampling twice, as %d and as %s)
    lines = ['Start Training...', 'init_step = %d' % init_step, 'batch_size = %d' % args.batch_size,
             'negative_adversarial_sampling = %d' % args.negative_adversarial_sampling,
             'hidden_dim = %d' % args.hidden_dim, 'gamma = %f' % args.gamma,
             'negative_adversarial_sampling = %s' % str(args.negative_adversarial_sampling)]
    if args.negative_adversarial_sampling:
        lines.append('adversarial_temperature = %f' % args.adversarial_temperature)
    for line in lines:
        logging.info(line)

    if args.do_train:
        logging.info('learning_rate = %d' % current_learning_rate)
        training_logs = []
        for step in range(init_step, args.max_steps):
            log = kge_model.train_step(kge_model, optimizer, train_iterator, args)
            training_logs.append(log)
            if step >= warm_up_steps:
                current_learning_rate = current_learning_rate / 10
                logging.info('Change learning_rate to %f at step %d' % (current_learning_rate, step))
                optimizer = KGEAdam(trainable(), lr=current_learning_rate)
                warm_up_steps = warm_up_steps * 3
            if step % args.save_checkpoint_steps == 0:
                osd = optimizer_state()
                full_table(True)
                if rank == 0:
                    save_model(kge_model, optimizer, {'step': step, 'current_learning_rate': current_learning_rate,
                                                      'warm_up_steps': warm_up_steps}, args, osd)
                full_table(False)
            if step % args.log_steps == 0:
                metrics = {}
                for metric in training_logs[0].keys():
                    metrics[metric] = sum([log[metric] for log in training_logs]) / len(training_logs)
                log_metrics('Training average', step, metrics)
                training_logs = []
            if args.do_valid and step % args.valid_steps == 0:
                full_table(True)
                if rank == 0:
                    logging.info('Evaluating on Valid Dataset...')
                    metrics = kge_model.test_step(kge_model, valid_triples, all_true_triples, args)
                    log_metrics('Valid', step, metrics)
                full_table(False)
        osd = optimizer_state()
        full_table(True)
        if rank == 0:
            save_model(kge_model, optimizer, {'step': step, 'current_learning_rate': current_learning_rate,
                                              'warm_up_steps': warm_up_steps}, args, osd)
    else:
        full_table(True)

    if rank != 0:
        return
    # final evaluations (the training split is logged under 'Test', as in the reference)
    for wanted, title, triples, label in ((args.do_valid, 'Valid', valid_triples, 'Valid'),
                                          (args.do_test, 'Test', test_triples, 'Test'),
                                          (args.evaluate_train, 'Training', train_triples, 'Test')):
        if wanted:
            logging.info('Evaluating on %s Dataset...' % title)
            log_metrics(label, step, kge_model.test_step(kge_model, triples, all_true_triples, args))


if __name__ == '__main__':
    main(parse_args())
