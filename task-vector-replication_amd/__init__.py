"""MI355X-native task-vector / function-vector engine.

Drop-in for the experiment path of IMMachinations/Task-Vector-Replication
(scratch.py / scratch2.py): the same experiment functions (``experiments``),
backed by a HIP/CDNA4 engine (``csrc/``, C ABI in ``include/tvr.h``) that runs
each sweep as one batched forward whose batch enumerates patch sites.

The directory name is not a Python identifier; import it through the
repository-root shim ``tvr_amd`` (``import tvr_amd``).
"""
from . import _lib, config, tasks, tokenizer, weights, prompts, model, experiments, distributed, results  # noqa: F401
from .config import PythiaConfig, get_config
from .model import Model, Trace, make_sites
from .results import load_results, save_results
from .experiments import (apply_layered_vectors_to_zero_shot, apply_layered_vectors_to_zero_shot_by_probability,
                          assemble_end_list_tasks, assemble_task_vector, calculate_average_causal_indirect_effect,
                          check_accuracy_of_added_task_vector, check_accuracy_of_task_vector,
                          gather_head_activations_to_layers, generate_mean_activation, generate_shuffled_prompt,
                          generate_shuffled_prompts, logits_to_next_k_tokens, substitute_task,
                          test_component_hypothesis)

__version__ = "0.1.0"
SUBMODULES = ("_lib", "config", "tasks", "tokenizer", "weights", "prompts", "model", "experiments",
              "distributed", "results")
