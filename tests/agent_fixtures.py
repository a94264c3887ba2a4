"""Shared scenario for the agent-loop parity test and its golden-vector generator
(tools/gen_golden_agent.py): an offline character-level tokenizer with a Qwen-style chat
template, a scripted inference client, and a small sqlite database. Pure data and plumbing:
nothing here is the code under test."""

import os
import sqlite3

CHAT_TEMPLATE = ("{% for m in messages %}<|im_start|>{{ m['role'] }}\n{{ m['content'] }}<|im_end|>\n{% endfor %}"
                 "{% if add_generation_prompt %}<|im_start|>assistant\n{% endif %}")
SPECIALS = ["<|endoftext|>", "<|im_start|>", "<|im_end|>"]


def make_tokenizer():
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast

    chars = [chr(c) for c in range(32, 127)] + ["\n", "\t"]
    vocab = {s: i for i, s in enumerate(SPECIALS + chars + ["<unk>"])}
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.Split(Regex(r"[\s\S]"), behavior="isolated")
    tk.decoder = decoders.Fuse()
    class ListChatTokenizer(PreTrainedTokenizerFast):
        # transformers 4.x behaviour (what the reference generator is written against):
        # apply_chat_template(tokenize=True) returns the id list, not a BatchEncoding
        def apply_chat_template(self, conversation, **kw):
            if kw.get("tokenize", True):
                kw.setdefault("return_dict", False)
            return super().apply_chat_template(conversation, **kw)

    t = ListChatTokenizer(tokenizer_object=tk, eos_token="<|im_end|>", pad_token="<|endoftext|>",
                          unk_token="<unk>", additional_special_tokens=SPECIALS)
    t.chat_template = CHAT_TEMPLATE
    return t


DB_ROWS = [(1, "alice", 34), (2, "bob", 27), (3, "carol", 41)]


def make_sql_root(root):
    """{root}/spider/database/people/people.sqlite with one table."""
    d = os.path.join(root, "spider", "database", "people")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "people.sqlite")
    if os.path.exists(path):
        os.remove(path)
    con = sqlite3.connect(path)
    con.execute("CREATE TABLE person (id INTEGER, name TEXT, age INTEGER)")
    con.executemany("INSERT INTO person VALUES (?, ?, ?)", DB_ROWS)
    con.commit()
    con.close()
    return root


# session -> scripted turns: (text, stop_reason, ends_with_eos)
SCRIPTS = {
    "sql_ok_0": [("<think>look up bob</think><sql>SELECT age FROM person WHERE name = 'bob'</sql>", "stop", False),
                 ("<think>it is 27</think><solution>SELECT age FROM person WHERE id = 2</solution>", "stop", False)],
    "sql_bad_0": [("<think>hmm</think> no tool call here", "stop", True),
                  ("<think>try</think><sql>SELECT nonexistent FROM person</sql>", "stop", False),
                  ("<think>guess</think><solution>SELECT 99</solution>", "stop", False)],
    "sql_turns_0": [("<think>a</think><sql>SELECT COUNT(*) FROM person</sql>", "stop", False),
                    ("<think>b</think><sql>SELECT MAX(age) FROM person</sql>", "stop", False),
                    ("<think>c</think><sql>SELECT MIN(age) FROM person</sql>", "stop", False)],
    "sql_fmt_0": [("<solution>SELECT age FROM person WHERE id = 2</solution>", "stop", False)],
    "sql_len_0": [("<think>" + "x" * 450 + "</think><sql>SELECT 1</sql>", "length", False)],
    "gsm_ok_0": [("6 * 7 = 42\n#### 42", "stop", True)],
    "gsm_bad_0": [("the answer is 41 #### 41", "stop", True)],
    "gsm_trunc_0": [("so far 4", "length", False)],
}


class ScriptedClient:
    """InferenceEngineClient stand-in: per session id, returns the next scripted turn (token ids
    through the shared tokenizer; eos appended when the script says the engine stopped on it)."""

    def __init__(self, tokenizer):
        self.tok = tokenizer
        self.turn = {}
        self.prompts = []

    async def generate(self, inp):
        sid = inp["session_ids"][0]
        k = self.turn.get(sid, 0)
        self.turn[sid] = k + 1
        text, reason, with_eos = SCRIPTS[sid][k]
        self.prompts.append((sid, list(inp["prompt_token_ids"][0])))
        ids = self.tok.encode(text, add_special_tokens=False)
        out_text = text
        if with_eos:
            ids = ids + [self.tok.eos_token_id]
            out_text = text + self.tok.eos_token
        lps = [-0.01 * (i + 1) for i in range(len(ids))]
        return {"responses": [out_text], "response_ids": [ids], "stop_reasons": [reason],
                "response_logprobs": [lps]}


def scenario(multi_turn):
    """GeneratorInput pieces (plain data) for one batch of 8 trajectories."""
    sys_msg = {"role": "system", "content": "Answer with SQL."}
    prompts, classes, extras, tids = [], [], [], []
    for name in ("sql_ok", "sql_bad", "sql_turns", "sql_fmt", "sql_len"):
        prompts.append([sys_msg, {"role": "user", "content": f"Task {name}: how old is bob?"}])
        classes.append("text2sql")
        extras.append({"db_id": "people", "data": "spider",
                       "reward_spec": {"ground_truth": "SELECT age FROM person WHERE name = 'bob'"}})
        tids.append((name, 0))
    for name, gt in (("gsm_ok", "42"), ("gsm_bad", "42"), ("gsm_trunc", "4")):
        prompts.append([{"role": "user", "content": f"{name}: what is 6*7?"}])
        classes.append("gsm8k")
        extras.append({"reward_spec": {"method": "rule", "ground_truth": gt}})
        tids.append((name, 0))
    return prompts, classes, extras, tids
