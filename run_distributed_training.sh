#!/bin/sh
# Multi-node launch (the reference's run_distributed_training.sh + Ansible
# playbook): write inv.yml from settings, rsync this directory to every node and
# start 8 ranks per node (one per MI355X) with node 0 as the rendezvous.
# Extra arguments go to train.py, e.g.  sh run_distributed_training.sh --epochs 10
DIR_IN=`pwd`
cd "$DIR_IN"
python create_inventory.py inv.yml
echo 'Created new inventory file based on settings'
exec python launch.py --hostfile inv.yml --workdir "$DIR_IN" --nproc_per_node "${GPUS_PER_NODE:-8}" -- train.py "$@"
