"""ProcessingStep / ProcessingPipeline — the reference's compose API
(pipeline.py:12-584), same constructor arguments, pairing modes, call
convention, logs and JSON dump, so a user pipeline built on the reference
runs unchanged with transforms from ``image_processor_pipeline_amd.transforms``.

Execution differs where the MI355X requires it (SURVEY §8b "Threading"):

* Transforms that drive the GPU are flagged ``fn.__ipp_device__ = True``.
  HIP state must not cross a ``fork``, so with ``workers > 1`` such a step runs
  in this (device-owning) process on a thread pool of ``workers`` threads —
  codec work (Pillow/zlib) releases the GIL, the kernels are stream-ordered.
  Plain Python plugins keep the reference's ``ProcessPoolExecutor``.
* A transform may expose ``fn.batch(list_of_arg_tuples, output_dirs=...,
  **options) -> list`` (one result or Exception per tuple, same order).  The
  step then hands it chunks of ``batch_size`` tuples so the pixel work of a
  chunk is one batched launch; per-item results are logged exactly as in the
  per-call path, and random draws happen in the same order.

Known reference defects fixed here: the parallel
branch increments an undefined ``errors_count`` (:429) — here it counts the
error; ``total_items`` for 'sample' calls ``min()`` (:279) — here it is the
input count; ``tqdm.notebook`` (:10) — here ``tqdm.auto``.
"""
from __future__ import annotations

import concurrent.futures
import json
import random
from collections import Counter
from os import cpu_count
from pathlib import Path
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple, Union
from warnings import warn

from tqdm.auto import tqdm

MODES = ('one_input', 'zip', 'modulo', 'sample', 'custom')

PathLike = Union[str, Path]


def _is_device_fn(fn: Callable) -> bool:
    return bool(getattr(fn, "__ipp_device__", False))


class ProcessingStep:
    """One transform applied to every input (tuple) of the step
    (reference pipeline.py:15-91)."""

    def __init__(self,
                 name: str,
                 process_function: Callable,
                 input_dirs: Optional[Union[PathLike, List[PathLike]]] = None,
                 output_dirs: Optional[Union[PathLike, List[PathLike]]] = None,
                 pairing_method: str = 'one_input',
                 pairing_function: Optional[Callable[[List[List[Path]]], Iterator[Tuple]]] = None,
                 fixed_input: bool = False,
                 root_dir: Optional[PathLike] = None,
                 sample_k: Optional[int] = None,
                 save_log: bool = False,
                 workers: Optional[int] = 1,
                 options: Optional[Dict] = None,
                 batch_size: int = 64):
        self.name = name
        self.process_function = process_function
        self.root_dir = Path(root_dir) if root_dir else None
        self.process_kwargs = options or {}
        self.sample_k = sample_k
        self.save_log = save_log
        self.batch_size = max(1, int(batch_size))

        self.input_paths: List[Path] = self._resolve_paths(input_dirs or [])
        self.output_paths: List[Path] = self._resolve_paths(output_dirs or [])
        self.fixed_input = fixed_input
        if not self.output_paths:
            raise ValueError(f"L'étape '{self.name}' doit avoir au moins un 'output_dirs' défini.")
        if pairing_method not in set(MODES):
            raise ValueError(f"Mode d'appariement' '{pairing_method}' invalide. Choisir parmi: {MODES}")
        if pairing_method == 'custom' and not callable(pairing_function):
            raise ValueError("Une `pairing_function` valide est requise pour le mode 'custom'.")
        self.pairing_method = pairing_method
        self.pairing_function = pairing_function
        self.process_logs: List[Dict[str, Any]] = []

        # workers: clamp to the machine, -1 = all cores (pipeline.py:84-90)
        max_cpus = cpu_count()
        if workers is not None and workers > max_cpus:
            warn(f"Nombre de workers parallèles ajusté à {max_cpus} (maximum système).")
        if workers == -1:
            workers = max_cpus
        self.parallels_workers = min(workers, max_cpus) if workers is not None else None

    def _resolve_paths(self, dir_list) -> List[Path]:
        """Relative entries are joined to root_dir when one is set (:92-111)."""
        items = dir_list if isinstance(dir_list, list) else [dir_list]
        out: List[Path] = []
        for folder in items:
            if not isinstance(folder, (str, Path)):
                raise ValueError(f"un élément ne représente pas un dossier ou un chemin : {folder}")
            p = Path(folder)
            out.append(self.root_dir / p if (self.root_dir and not p.is_absolute()) else p)
        return out

    def __str__(self) -> str:
        ins = ", ".join(p.name for p in self.input_paths)
        outs = ", ".join(p.name for p in self.output_paths)
        return (f"Étape '{self.name}':\n"
                f"  Entrée(s) : [{ins}] (Mode: {self.pairing_method})\n"
                f"  Sortie(s) : [{outs}]\n"
                f"  Options   : {self.process_kwargs}")

    # ---------------------------------------------------------------- inputs
    def _get_files_from_inputs(self) -> List[List[Path]]:
        """Sorted regular files of every input dir (:122-146)."""
        if not self.input_paths:
            raise ValueError(f"{self.name} : Aucun dossier d'entrée défini.")
        print(f"Info [{self.name}]: Récupération des chemins de fichiers d'entrée...")
        lists = []
        for d in self.input_paths:
            if not d.is_dir():
                raise FileNotFoundError(
                    f"Le dossier d'entrée spécifié n'existe pas: '{d}' pour l'étape '{self.name}'")
            try:
                files = sorted(f for f in d.iterdir() if f.is_file())
            except Exception as e:
                raise IOError(f"Échec de l'inventaire du dossier {d}") from e
            print(f"  '{d.name}' : {len(files)} fichiers trouvés.")
            lists.append(files)
        return lists

    def _generate_processing_inputs(self, input_file_lists: List[List[Path]]) -> Iterator[Tuple]:
        """Argument tuples per pairing mode (:148-235); random draws in the
        reference's order (sample_k, modulo shuffle, sample's two draws)."""
        n_lists = len(input_file_lists)
        if not all(input_file_lists):
            empty = [str(self.input_paths[i]) for i, lst in enumerate(input_file_lists) if not lst]
            raise FileNotFoundError(f"Aucun fichier trouvé dans les dossiers d'entrée {empty} pour l'étape '{self.name}'.")
        if self.sample_k and isinstance(self.sample_k, int):
            ids = random.sample(range(len(input_file_lists[0])), self.sample_k)
            input_file_lists = [[lst[i] for i in ids] for lst in input_file_lists]

        mode = self.pairing_method
        if mode == 'one_input':
            if n_lists == 0:
                raise ValueError("Mode 'one_input' mais aucun dossier d'entrée fourni.")
            for f in input_file_lists[0]:
                yield (f,)
        elif mode == 'zip':
            if n_lists < 2:
                raise ValueError("Le mode 'zip' requiert au moins 2 dossiers d'entrée.")
            yield from zip(*input_file_lists)
        elif mode == 'modulo':
            if n_lists != 2:
                raise ValueError("Le mode 'modulo' requiert exactement 2 dossiers d'entrée.")
            first, second = input_file_lists
            random.shuffle(second)
            for i, p in enumerate(first):
                yield (p, second[i % len(second)])
        elif mode == 'sample':
            files = input_file_lists[0]
            blur = set(random.sample(files, int(len(files) * 0.3)))
            rgb = set(random.sample(files, int(len(files) * 0.3)))
            yield from zip(files, [f in blur for f in files], [f in rgb for f in files])
        elif mode == 'custom':
            if not self.pairing_function:
                raise ValueError("Fonction `pairing_function` manquante pour le mode 'custom'.")
            yield from self.pairing_function(input_file_lists)
        else:
            raise NotImplementedError(f"Mode d'appariement' '{mode}' non implémentée.")

    # ------------------------------------------------------------------- run
    def run(self):
        """Create output dirs, list inputs, process, log (:237-302)."""
        self.process_logs = []
        print(f"--- Exécution Étape : {self.name} ---")
        print(f"Info [{self.name}]: Vérification/Création des dossiers de sortie...")
        for out in self.output_paths:
            try:
                out.mkdir(parents=True, exist_ok=True)
                print(f"  Sortie -> '{out}'")
            except IOError as ioe:
                raise IOError(f"Impossible de créer le dossier de sortie '{out}': {ioe}") from ioe
            except Exception as e:
                print(f"Erreur lors de la création du dossier {out}. {e}")
                return
        try:
            lists = self._get_files_from_inputs()
        except (FileNotFoundError, ValueError, IOError) as e:
            print(f"Erreur [{self.name}]: Condition préalable non remplie pour démarrer l'étape. {e}")
            return
        try:
            args_iter = self._generate_processing_inputs(lists)
        except (ValueError, NotImplementedError) as e:
            print(f"Erreur [{self.name}]: Impossible de générer les arguments pour le mode '{self.pairing_method}'. {e}")
            return

        total = None
        if self.pairing_method in ('one_input', 'modulo', 'sample'):
            total = self.sample_k if (self.sample_k and isinstance(self.sample_k, int)) else len(lists[0])
        elif self.pairing_method == 'zip':
            total = min(len(lst) for lst in lists)

        processed, errors = self._processing_loop(args_iter, total)
        if self.process_logs and self.save_log:
            self._save_process_logs_to_json()
        else:
            print(f"Info [{self.name}] : Aucun log de traitement généré.")
        print(f"--- Étape {self.name} terminée ---")
        print(f"  {processed} éléments traités avec succès (fichiers de sortie générés).")
        if errors > 0:
            print(f"  {errors} erreur(s) ou traitement(s) sans retour.")

    @staticmethod
    def _new_log(args: Tuple, status: str) -> Dict[str, Any]:
        return {"inputs": list(args), "outputs": None, "status": status, "error_message": None}

    def _record(self, log: Dict[str, Any], result: Any, exc: Optional[BaseException], err_prefix: str) -> bool:
        if exc is not None:
            msg = f"{err_prefix}{exc}"
            tqdm.write(f"\nErreur [{self.name}]: {msg}")
            log.update({"status": "Error", "error_message": msg if err_prefix else str(exc)})
            ok = False
        else:
            ok = self._build_log(log, result)
        self.process_logs.append(log)
        return ok

    def _processing_loop(self, argument_iterator: Iterator[Tuple], total_items: Optional[int]) -> Tuple[int, int]:
        """Sequential, batched, threaded (device) or process-pool execution
        (:304-437).  Returns (success_count, error_count)."""
        fn = self.process_function
        workers = self.parallels_workers
        sequential = not workers or 0 <= workers <= 1
        batch = getattr(fn, "batch", None)
        ok_n = err_n = 0
        bar = dict(desc=self.name, unit="item", leave=True, smoothing=0)

        if batch is not None and callable(batch):
            print(f"Info [{self.name}]: Exécution par lots de {self.batch_size} (GPU)...")
            with tqdm(total=total_items, **bar) as pbar:
                chunk: List[Tuple] = []
                for args in list(argument_iterator) + [None]:
                    if args is not None:
                        chunk.append(args)
                        if len(chunk) < self.batch_size:
                            continue
                    if not chunk:
                        break
                    try:
                        results = batch(chunk, output_dirs=self.output_paths, threads=max(1, workers or 1),
                                        **self.process_kwargs)
                        if len(results) != len(chunk):
                            raise RuntimeError(f"batch returned {len(results)} results for {len(chunk)} inputs")
                    except Exception as e:   # the whole chunk failed
                        results = [e] * len(chunk)
                    for a, r in zip(chunk, results):
                        exc = r if isinstance(r, BaseException) else None
                        good = self._record(self._new_log(a, "Pending"), None if exc else r, exc,
                                            f"Échec traitement de {a}: " if exc else "")
                        ok_n += good
                        err_n += not good
                    pbar.update(len(chunk))
                    chunk = []
            return ok_n, err_n

        if sequential:
            print(f"Info [{self.name}]: Exécution en mode séquentiel...")
            for args in tqdm(argument_iterator, total=total_items, **bar):
                log = self._new_log(args, "Pending")
                try:
                    res = fn(*args, output_dirs=self.output_paths, **self.process_kwargs)
                    good = self._record(log, res, None, "")
                except Exception as e:
                    tqdm.write(f"\nErreur [{self.name}]: Échec traitement de {args}: {e}")
                    log.update({"status": "Error", "error_message": str(e)})
                    self.process_logs.append(log)
                    good = False
                ok_n += good
                err_n += not good
            return ok_n, err_n

        if workers > 1:
            device = _is_device_fn(fn)
            print(f"Info [{self.name}]: Exécution en mode parallèle avec {workers} workers"
                  f"{' (threads, processus GPU)' if device else ''}...")
            arg_list = list(argument_iterator)
            if not arg_list:
                raise RuntimeError("Aucun argument à traiter après génération. Fin.")
            pool_cls = concurrent.futures.ThreadPoolExecutor if device else concurrent.futures.ProcessPoolExecutor
            with pool_cls(max_workers=workers) as ex:
                fut_to_log: Dict[concurrent.futures.Future, Dict[str, Any]] = {}
                print(f"Info [{self.name}]: Soumission de {len(arg_list)} tâches au pool de processus...")
                for args in arg_list:
                    log = self._new_log(args, "Pending Execution")
                    try:
                        fut_to_log[ex.submit(fn, *args, output_dirs=self.output_paths, **self.process_kwargs)] = log
                    except Exception as e:
                        tqdm.write(f"Erreur [{self.name}]: Échec de la soumission de la tâche pour {args}: {e}")
                        log.update({"status": "Submission Error", "error_message": str(e)})
                        self.process_logs.append(log)
                        err_n += 1
                for fut in tqdm(concurrent.futures.as_completed(fut_to_log), total=len(fut_to_log), **bar):
                    log = fut_to_log[fut]
                    try:
                        res = fut.result()
                        good = self._record(log, res, None, "")
                    except Exception as e:
                        prefix = f"Échec tâche parallèle pour {[str(p) for p in log['inputs']]} : "
                        good = self._record(log, None, e, prefix)
                    ok_n += good
                    err_n += not good
            return ok_n, err_n
        raise ValueError("Logique non prévue, veuillez revoir le nombre de workers attribués à la tâche.")

    def _build_log(self, log_entry: Dict[str, Any], saved_output_paths: Any) -> bool:
        """Success for a Path or a list of Paths; 'Type Error' for any other
        truthy value; 'no_output' for None/falsy (:439-470)."""
        if not saved_output_paths:
            log_entry["status"] = "no_output"
            return False
        if isinstance(saved_output_paths, Path):
            log_entry.update({"outputs": [saved_output_paths], "status": "Success"})
            return True
        if isinstance(saved_output_paths, list) and all(isinstance(p, Path) for p in saved_output_paths):
            log_entry.update({"outputs": saved_output_paths, "status": "Success"})
            return True
        name = getattr(self.process_function, "__name__", repr(self.process_function))
        msg = (f"Retour invalide (parallèle) de {name} pour {[str(p) for p in log_entry['inputs']]} "
               f"(type : {type(saved_output_paths)}).Attendu Path, List[Path] ou None.")
        warn(msg)
        log_entry.update({"status": "Type Error", "error_message": msg})
        return False

    def _save_process_logs_to_json(self) -> None:
        """``output_paths[0].parent / f"{name}.json"`` (:472-499)."""
        if not self.output_paths:
            warn(f"Avertissement [{self.name}] : Aucun dossier de sortie configuré."
                 "Enregistrement du mappage des fichiers impossible.")
            return
        if not self.process_logs:
            print(f"Info [{self.name}] : Aucun fichier traité à enregistrer dans le JSON (`process_logs` est vide).")
            return
        path = self.output_paths[0].parent / Path(self.name).with_suffix(".json")
        print(f"Info [{self.name}]: Enregistrement des logs de fichiers traités dans {path}...")
        try:
            with path.open("w", encoding="utf-8") as fh:
                json.dump(self.process_logs, fh, indent=4, ensure_ascii=False, cls=PathJSONEncoder)
            print(f"Info [{self.name}]: Logs sauvegardé avec succès.")
        except (IOError, TypeError) as e:
            print(f"Erreur critique [{self.name}]: Impossible d'enregistrer le fichier JSON des résultats: {e}")
        except Exception as e:
            print(f"Erreur inattendue [{self.name}] lors de la sauvegarde JSON: {e}")


class ProcessingPipeline:
    """Ordered steps with output→input chaining (reference :502-566)."""

    def __init__(self, root_dir: Optional[PathLike] = None):
        self.steps: List[ProcessingStep] = []
        self.root_dir = Path(root_dir) if root_dir else None

    def add_step(self, step: ProcessingStep, position=None):
        if not self.steps and not step.input_paths:
            raise ValueError(f"La première étape ('{step.name}') doit avoir `input_dirs` définie.")
        if self.root_dir and not step.root_dir:
            step.root_dir = self.root_dir
            step.input_paths = step._resolve_paths(step.input_paths)
            step.output_paths = step._resolve_paths(step.output_paths)
        position = len(self.steps) if position is None else position
        if not step.input_paths:
            if position == 0:
                raise IndexError(f"Insertion en première position, impossible de déduire les dossiers d'input pour {step.name}")
            try:
                prev = self.steps[position - 1]
                nxt = self.steps[position] if position < len(self.steps) else None
                step.input_paths = prev.output_paths
                if nxt and not nxt.fixed_input:
                    nxt.input_paths = step.output_paths
            except IndexError as idx:
                raise ValueError(f"Position d'insertion invalide pour déduire les dossiers d'input de {step.name}.") from idx
            except Exception as e:
                raise RuntimeError(f"Erreur inattendue pour l'ajout de {step.name}") from e
        self.steps.insert(position, step)

    def run(self, from_step_index: int = 0, only_one: bool = False):
        if from_step_index < 0 or from_step_index >= len(self.steps):
            raise IndexError(f"Invalid start index {from_step_index}. Pipeline has {len(self.steps)} steps.")
        todo = [self.steps[from_step_index]] if only_one else self.steps[from_step_index:]
        for i, step in enumerate(todo, start=from_step_index):
            print(f"Running étape {i}: {step.name}")
            step.run()


class PathJSONEncoder(json.JSONEncoder):
    """Paths → str, tuples → lists (reference :569-584)."""

    def default(self, o: Any) -> Any:
        if isinstance(o, Path):
            return str(o)
        if isinstance(o, tuple):
            return list(o)
        return super().default(o)
