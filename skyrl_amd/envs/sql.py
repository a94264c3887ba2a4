"""SkyRL-SQL environment (config 5): multi-turn text-to-SQL with an sqlite tool.

Restates skyrl_gym/envs/sql/env.py:17-148 (turn accounting, `<sql>` tool calls, observations
as user messages, reward only at the end), the tool skyrl_gym/tools/sql.py:9-93 (read-only
execution in a rolled-back transaction with a timeout, rows as a frozenset rendered by pandas,
the `<observation>...<reminder>` wrapper) and the reward skyrl_gym/envs/sql/utils.py:17-133
(format check -> -1, result-set equality with the gold query -> 1, else 0).
"""

from __future__ import annotations

import os
import re
import sqlite3
import threading
from typing import Any, Dict, Optional, Tuple

from .base import BaseTextEnv, BaseTextEnvStepOutput, register

_TASK_DIRS = {"synsql": "SynSQL-2.5M/databases", "spider": "spider/database", "bird": "bird/train/train_databases"}
_INVALID_ACTION = ("Your previous action is invalid. Follow the format of outputting thinking process and sql tool, "
                   "and try again.")


def _run_sql(db_file: str, sql: str, timeout: float):
    """(rows frozenset | None, error text | None, timed_out). Read-only: the transaction is rolled
    back; a query past `timeout` seconds is interrupted."""
    box: Dict[str, Any] = {"rows": None, "err": None, "conn": None}
    finished = threading.Event()

    def work():
        conn = None
        try:
            conn = sqlite3.connect(db_file, check_same_thread=False)
            box["conn"] = conn
            cur = conn.cursor()
            conn.execute("BEGIN TRANSACTION;")
            cur.execute(sql)
            box["rows"] = frozenset(cur.fetchall())
        except Exception as e:  # noqa: BLE001 - reported to the model as the observation
            box["err"] = e
        finally:
            if conn is not None:
                try:
                    conn.rollback()
                except Exception:  # noqa: BLE001
                    pass
                try:
                    conn.close()
                except Exception:  # noqa: BLE001
                    pass
            finished.set()

    threading.Thread(target=work, daemon=True).start()
    timed_out = False
    if not finished.wait(timeout):
        timed_out = True
        if box["conn"] is not None:
            try:
                box["conn"].interrupt()
            except Exception:  # noqa: BLE001
                pass
        finished.wait()
    return box["rows"], box["err"], timed_out


def sql_tool_observation(db_file: str, sql: Optional[str], turns_left: int, timeout: float = 5) -> str:
    """The tool message the model sees after a `<sql>` call (tools/sql.py)."""
    if sql is None:
        obs = _INVALID_ACTION
    else:
        rows, err, timed_out = _run_sql(db_file, sql, timeout)
        if timed_out:
            obs = f"SQL Timeout:\n{sql}"
        elif rows is None:
            obs = f"Error executing SQL: {err}, db file: {db_file}"
        else:
            import pandas as pd

            df = pd.DataFrame(rows)
            obs = df.to_string(index=False)
            if len(obs) > 9000:
                obs = "Truncated to 50 lines since returned response too long: " + df.head(50).to_string(index=False)
    reminder = f"<reminder>You have {turns_left} turns left to complete the task.</reminder>"
    return f"\n\n<observation>{obs}\n{reminder}</observation>\n\n"


def verify_format_and_extract(output: str) -> Tuple[bool, Optional[list], Optional[str]]:
    """One <solution> block, no think/sql/observation tags inside it, at least one <think>, and
    every </observation> followed by a <think> (utils.py:17-44)."""
    if output.count("<solution>") != 1:
        return False, None, None
    pre, tail = output.split("<solution>", 1)
    if tail.count("</solution>") != 1:
        return False, None, None
    solution = tail.split("</solution>", 1)[0]
    if re.search(r"</?(think|sql|observation)\b", solution, re.I):
        return False, None, None
    thoughts = re.findall(r"<think>(.*?)</think>", output, re.S)
    if not thoughts:
        return False, None, None
    for m in re.finditer(r"</observation>", pre, re.I):
        if not pre[m.end():].lstrip().lower().startswith("<think>"):
            return False, None, None
    return True, thoughts, solution.strip()


def compute_score_single(completion: str, gold_sql: str, db_file: str, timeout: float = 30) -> float:
    try:
        ok, _, pred_sql = verify_format_and_extract(completion)
        if not ok:
            return -1.0
        pred, _, _ = _run_sql(db_file, pred_sql, timeout)
        gold, _, _ = _run_sql(db_file, gold_sql, timeout)
        return 1.0 if (pred is not None and gold is not None and pred == gold) else 0.0
    except Exception:  # noqa: BLE001 - the reference scores unexpected failures as 0
        return 0


class SQLEnv(BaseTextEnv):
    def __init__(self, env_config: Any = None, extras: Dict[str, Any] = None):
        super().__init__()
        extras = extras or {}
        for k in ("db_id", "reward_spec", "data"):
            if k not in extras:
                raise ValueError(f"text2sql needs extras[{k!r}]")
        root = env_config.get("db_path") if isinstance(env_config, dict) else getattr(env_config, "db_path", None)
        if extras["data"] not in _TASK_DIRS:
            raise NotImplementedError(f"unknown text2sql task {extras['data']!r}")
        self.db_id = extras["db_id"]
        self.gold_sql = extras["reward_spec"]["ground_truth"]
        self.db_dir = os.path.join(root or "", _TASK_DIRS[extras["data"]])
        self.db_file = os.path.join(self.db_dir, self.db_id, self.db_id + ".sqlite")
        if not os.path.exists(self.db_file):
            raise FileNotFoundError(f"Database file not found at: {self.db_file}")
        self.max_turns = extras.get("max_turns", 5)
        self.chat_history = []

    def step(self, action: str) -> BaseTextEnvStepOutput:
        self.turns += 1
        for tag in ("</sql>", "</solution>"):  # stop strings end the action (env.py:96-103)
            if tag in action and action.split(tag, 1)[1] != "":
                raise AssertionError(f"{tag} detected in the response but it is not the last string generated.")
        self.chat_history.append({"role": "assistant", "content": action})
        done = self.turns >= self.max_turns or ("<solution>" in action and "</solution>" in action)
        if done:
            text = "".join(m["content"] for m in self.chat_history)
            return BaseTextEnvStepOutput(observations=[], reward=compute_score_single(text, self.gold_sql, self.db_file),
                                         done=True, metadata={})
        m = re.search(r"<sql>(.*?)</sql>", action, re.DOTALL)
        sql = m.group(1) if m else None
        try:
            obs = sql_tool_observation(self.db_file, sql, self.max_turns - self.turns)
            info = {"tool_group": "SQLCodeExecutorToolGroup", "tool_name": "sql",
                    "tool_input": (self.db_id, sql, self.max_turns - self.turns)}
        except Exception as e:  # noqa: BLE001
            obs = str(e)
            info = {"tool_group": None, "tool_name": None, "tool_input": ""}
        new_obs = {"role": "user", "content": obs} if obs else None
        if new_obs:
            self.chat_history.append(new_obs)
        return BaseTextEnvStepOutput(observations=[new_obs] if new_obs else [], reward=0, done=False, metadata=info)


register("text2sql", SQLEnv)
