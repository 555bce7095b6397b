from .zoo import (ClientFront, ClientFrontSisa, ServerTailUShape, ServerTailSisa,
                  ServerTailSisaConcat, Head, LinearSpec, TailSpec, ushape_server_spec,
                  sisa_server_spec, head_spec, model1, model1_sisa, model2, model2_sisa,
                  model2_sisa_concat, model3)

__all__ = ["ClientFront", "ClientFrontSisa", "ServerTailUShape", "ServerTailSisa",
           "ServerTailSisaConcat", "Head", "LinearSpec", "TailSpec", "ushape_server_spec",
           "sisa_server_spec", "head_spec", "model1", "model1_sisa", "model2", "model2_sisa",
           "model2_sisa_concat", "model3"]
