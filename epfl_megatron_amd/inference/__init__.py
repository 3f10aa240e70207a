"""Text generation / scoring / beam search and the REST server
(reference ``megatron/text_generation`` and ``megatron/text_generation_server.py``)."""
from .api import (beam_search, beam_search_and_post_process, generate,  # noqa: F401
                  generate_and_post_process)
